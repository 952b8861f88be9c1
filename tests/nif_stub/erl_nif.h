/* Declaration stub of the OTP erl_nif API subset emqx_amd/csrc/emqx_trie_nif.c
 * uses (signatures as documented for OTP 21+, erl_nif(3)).  TEST
 * INFRASTRUCTURE ONLY: it lets tests/test_nif_build.py compile the NIF shim
 * with -fsyntax-only -Werror in this image, which has no Erlang/OTP.  It is
 * not linked, not loaded and not a runtime stand-in for OTP. */
#ifndef TM_TEST_ERL_NIF_STUB_H
#define TM_TEST_ERL_NIF_STUB_H
#include <stddef.h>
#include <stdint.h>

typedef uintptr_t ERL_NIF_TERM;
typedef uint64_t ErlNifUInt64;
typedef struct enif_environment_t ErlNifEnv;
typedef struct enif_resource_type_t ErlNifResourceType;
typedef void ErlNifResourceDtor(ErlNifEnv*, void*);
typedef enum { ERL_NIF_RT_CREATE = 1, ERL_NIF_RT_TAKEOVER = 2 } ErlNifResourceFlags;
typedef enum { ERL_NIF_LATIN1 = 1 } ErlNifCharEncoding;
#define ERL_NIF_DIRTY_JOB_CPU_BOUND 1
#define ERL_NIF_DIRTY_JOB_IO_BOUND 2

typedef struct {
    size_t size;
    unsigned char* data;
    void* ref_bin;
    void* __spare__[2];
} ErlNifBinary;
typedef struct {
    ERL_NIF_TERM pid;
} ErlNifPid;
typedef struct {
    const char* name;
    unsigned arity;
    ERL_NIF_TERM (*fptr)(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]);
    unsigned flags;
} ErlNifFunc;

int enif_make_existing_atom(ErlNifEnv*, const char*, ERL_NIF_TERM*, ErlNifCharEncoding);
ERL_NIF_TERM enif_make_atom(ErlNifEnv*, const char*);
ERL_NIF_TERM enif_make_atom_len(ErlNifEnv*, const char*, size_t);
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_tuple5(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_badarg(ErlNifEnv*);
ErlNifResourceType* enif_open_resource_type(ErlNifEnv*, const char*, const char*, ErlNifResourceDtor*,
                                            ErlNifResourceFlags, ErlNifResourceFlags*);
int enif_get_resource(ErlNifEnv*, ERL_NIF_TERM, ErlNifResourceType*, void**);
void* enif_alloc_resource(ErlNifResourceType*, size_t);
void enif_release_resource(void*);
void enif_keep_resource(void*);
ERL_NIF_TERM enif_make_resource(ErlNifEnv*, void*);
int enif_get_int(ErlNifEnv*, ERL_NIF_TERM, int*);
int enif_inspect_binary(ErlNifEnv*, ERL_NIF_TERM, ErlNifBinary*);
unsigned char* enif_make_new_binary(ErlNifEnv*, size_t, ERL_NIF_TERM*);
void* enif_alloc(size_t);
void enif_free(void*);
ERL_NIF_TERM enif_make_list(ErlNifEnv*, unsigned, ...);
ERL_NIF_TERM enif_make_list1(ErlNifEnv*, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_list_from_array(ErlNifEnv*, const ERL_NIF_TERM[], unsigned);
ERL_NIF_TERM enif_make_uint(ErlNifEnv*, unsigned);
ERL_NIF_TERM enif_make_uint64(ErlNifEnv*, ErlNifUInt64);
int enif_get_list_cell(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM*, ERL_NIF_TERM*);
int enif_get_list_length(ErlNifEnv*, ERL_NIF_TERM, unsigned*);
int enif_is_binary(ErlNifEnv*, ERL_NIF_TERM);
int enif_is_atom(ErlNifEnv*, ERL_NIF_TERM);
int enif_is_list(ErlNifEnv*, ERL_NIF_TERM);
int enif_is_identical(ERL_NIF_TERM, ERL_NIF_TERM);
int enif_send(ErlNifEnv*, const ErlNifPid*, ErlNifEnv*, ERL_NIF_TERM);
ErlNifEnv* enif_alloc_env(void);
void enif_free_env(ErlNifEnv*);
ERL_NIF_TERM enif_make_ref(ErlNifEnv*);
ERL_NIF_TERM enif_make_copy(ErlNifEnv*, ERL_NIF_TERM);
ErlNifPid* enif_self(ErlNifEnv*, ErlNifPid*);

typedef struct {
    const char* name;
    ErlNifFunc* funcs;
    int (*load)(ErlNifEnv*, void**, ERL_NIF_TERM);
    int (*reload)(ErlNifEnv*, void**, ERL_NIF_TERM);
    int (*upgrade)(ErlNifEnv*, void**, void**, ERL_NIF_TERM);
    void (*unload)(ErlNifEnv*, void*);
} ErlNifEntryStub;
#define ERL_NIF_INIT(NAME, FUNCS, LOAD, RELOAD, UPGRADE, UNLOAD)                   \
    const ErlNifEntryStub* nif_init(void);                                       \
    const ErlNifEntryStub* nif_init(void) {                                      \
        static ErlNifEntryStub entry = {#NAME, FUNCS, LOAD, RELOAD, UPGRADE, UNLOAD}; \
        return &entry;                                                           \
    }
#endif

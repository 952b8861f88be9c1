%% emqx_trie_nif — loader of the GPU topic-routing NIF (emqx_amd/csrc/emqx_trie_nif.c
%% over libtopicmatch, include/topicmatch.h).  Every function below is replaced
%% by its NIF on load; the bodies only run when the library is missing.
%%
%% Install: copy libtopicmatch.so and emqx_trie_nif.so (make nif
%% ERL_INCLUDE=...) into emqx's priv dir.
-module(emqx_trie_nif).

-export([open/1, insert/2, delete/2, lookup/2, commit/1, match/2, match_many/2,
         match_async/2, match_routes_async/2, match_deliveries_async/2,
         dest_target/4, route_add/3, route_del/3, route_write/3, route_delete_object/3]).

-on_load(init/0).

init() ->
    Priv = case code:priv_dir(emqx) of
               {error, bad_name} -> "priv";
               Dir -> Dir
           end,
    erlang:load_nif(filename:join(Priv, "emqx_trie_nif"), 0).

%% open(Device | [Device]) -> {ok, Engine} | {error, Reason}
open(_Devices) -> erlang:nif_error(nif_not_loaded).
%% emqx_trie:insert/1, delete/1 (src/emqx_trie.erl:62-73, 88-96)
insert(_Engine, _Filter) -> erlang:nif_error(nif_not_loaded).
delete(_Engine, _Filter) -> erlang:nif_error(nif_not_loaded).
%% emqx_trie:lookup/1 (src/emqx_trie.erl:83-84): [] | [#trie_node{}], i.e.
%% [{trie_node, NodeId, EdgeCount, Topic | undefined, undefined}] (include/emqx.hrl:95-100)
lookup(_Engine, _NodeId) -> erlang:nif_error(nif_not_loaded).
commit(_Engine) -> erlang:nif_error(nif_not_loaded).
%% emqx_trie:match/1 (src/emqx_trie.erl:77-79), synchronous on a dirty IO scheduler
match(_Engine, _Topic) -> erlang:nif_error(nif_not_loaded).
match_many(_Engine, _Topics) -> erlang:nif_error(nif_not_loaded).
%% micro-batched: return Ref at once, the reply {Ref, Result} arrives later
match_async(_Engine, _Topic) -> erlang:nif_error(nif_not_loaded).
match_routes_async(_Engine, _Topic) -> erlang:nif_error(nif_not_loaded).
match_deliveries_async(_Engine, _Topic) -> erlang:nif_error(nif_not_loaded).
%% aggre/1 target of a dest: node (the atom's text) or group (the Group binary)
dest_target(_Engine, _DestBin, _Kind, _Key) -> erlang:nif_error(nif_not_loaded).
%% emqx_router add/del route (src/emqx_router.erl:153-187, 226-260)
route_add(_Engine, _Topic, _DestBin) -> erlang:nif_error(nif_not_loaded).
route_del(_Engine, _Topic, _DestBin) -> erlang:nif_error(nif_not_loaded).
%% the emqx_route table events (emqx_trie_gpu_feed): the route bag only, never
%% the trie -- mnesia:write / mnesia:delete_object of #route{}
%% (src/emqx_router.erl:223-224, 231, 240-241, 255-257; emqx_router_helper.erl:156-160)
route_write(_Engine, _Topic, _DestBin) -> erlang:nif_error(nif_not_loaded).
route_delete_object(_Engine, _Topic, _DestBin) -> erlang:nif_error(nif_not_loaded).

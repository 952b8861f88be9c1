%% emqx_trie_gpu — the GPU-backed forms of the hot-path functions, with the
%% reference's names, arities and return shapes:
%%
%%   match/1           = emqx_trie:match/1           (src/emqx_trie.erl:77-79)
%%   lookup/1          = emqx_trie:lookup/1          (src/emqx_trie.erl:83-84)
%%   match_routes/1    = emqx_router:match_routes/1  (src/emqx_router.erl:116-118)
%%   match_deliveries/1 = emqx_broker:aggre(emqx_router:match_routes(T))
%%                                                  (src/emqx_broker.erl:152, 194-206)
%%
%% A call submits the topic to the engine's micro-batcher and waits for its
%% own reply (the batcher seals device batches across all publishing
%% processes; nothing blocks a scheduler).  The engine handle lives in the
%% public ETS table ?TAB, written once by emqx_trie_gpu_feed at boot (OTP 21.0
%% has no persistent_term).  Usage in the reference:
%%
%%   emqx_trie:match(Topic)          -> emqx_trie_gpu:match(Topic)
%%   emqx_router:match_routes(Topic) -> emqx_trie_gpu:match_routes(Topic)
%%   emqx_broker:publish/1:  route(aggre(match_routes(Topic)), D)
%%                        -> route(emqx_trie_gpu:match_deliveries(Topic), D)
-module(emqx_trie_gpu).

-include_lib("emqx/include/emqx.hrl").

-export([engine/0, match/1, lookup/1, match_routes/1, match_deliveries/1, match_many/1]).

-define(TAB, emqx_trie_gpu).
-define(TIMEOUT, 5000).
-define(LATE, emqx_trie_gpu_late).   %% process dictionary: refs of replies that timed out

engine() ->
    [{engine, E}] = ets:lookup(?TAB, engine),
    E.

%% emqx_trie:match/1: [Filter] in the reference's order
match(Topic) when is_binary(Topic) ->
    wait(emqx_trie_nif:match_async(engine(), Topic)).

%% emqx_trie:lookup/1: [] | [#trie_node{}] from the engine's host mirror
%% (edge_count and topic kept exactly as emqx_trie:insert/1, delete/1 keep them)
lookup(NodeId) when is_binary(NodeId) ->
    case emqx_trie_nif:lookup(engine(), NodeId) of
        {error, _} = E -> error(E);
        Nodes -> Nodes
    end.

%% many topics in one device batch (print_routes, tests, bulk callers)
match_many(Topics) when is_list(Topics) ->
    case emqx_trie_nif:match_many(engine(), Topics) of
        {error, _} = E -> error(E);
        Lists -> Lists
    end.

%% emqx_router:match_routes/1: [#route{}] — the literal topic's routes first,
%% then each matched filter's, in trie order
match_routes(Topic) when is_binary(Topic) ->
    [#route{topic = To, dest = binary_to_term(D)}
     || {To, D} <- wait(emqx_trie_nif:match_routes_async(engine(), Topic))].

%% aggre(match_routes(Topic)): [{To, Node} | {To, Group}] in aggre/1's order
match_deliveries(Topic) when is_binary(Topic) ->
    wait(emqx_trie_nif:match_deliveries_async(engine(), Topic)).

wait({error, _} = E) ->
    error(E);
wait(Ref) when is_reference(Ref) ->
    flush_late(),
    receive
        {Ref, {error, _} = E} -> error(E);
        {Ref, Result} -> Result
    after ?TIMEOUT ->
        %% the batcher still answers this Ref later: drop the reply if it
        %% came in the meantime, else remember the Ref so that the caller's
        %% next wait/1 drops it (OTP 21 has no aliases to cancel a reply)
        receive
            {Ref, _} -> ok
        after 0 ->
            put(?LATE, [Ref | late()])
        end,
        error({emqx_trie_gpu, timeout})
    end.

late() ->
    case get(?LATE) of
        undefined -> [];
        L -> L
    end.

%% drop the late replies that have arrived; keep waiting for the others
flush_late() ->
    case late() of
        [] -> ok;
        L ->
            case [R || R <- L, not drop(R)] of
                [] -> erase(?LATE);
                Rest -> put(?LATE, Rest)
            end,
            ok
    end.

drop(Ref) ->
    receive
        {Ref, _} -> true
    after 0 ->
        false
    end.

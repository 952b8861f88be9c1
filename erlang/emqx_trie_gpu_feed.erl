%% emqx_trie_gpu_feed — keeps the GPU engine's image equal to the committed
%% mnesia state (SURVEY H4).  A child of emqx_sup next to emqx_router_sup
%% (src/emqx_sup.erl:57-88):
%%
%%   {emqx_trie_gpu_feed, {emqx_trie_gpu_feed, start_link, []},
%%    permanent, 5000, worker, [emqx_trie_gpu_feed]}
%%
%% At boot it opens the engine on the GPUs of app env {emqx, trie_gpu_devices}
%% (an integer or a list; default [0]), subscribes to the detailed events of
%% both tables, and only THEN loads their current contents: a write committed
%% between the two steps is in the snapshot and also queued as an event, and
%% every handler below is an idempotent set operation, so replaying the queued
%% events over the snapshot ends in the committed state (the other order loses
%% such a write until restart).  Local transactions (emqx_router
%% add/del_trie_route, src/emqx_router.erl:226-260) and writes replicated from
%% other nodes (src/emqx_trie.erl:50-54) arrive the same way, after commit,
%% so an aborted transaction never reaches the image.
%%
%% The two tables drive two independent things, exactly as in the reference:
%%   emqx_trie_node events -> trie membership (emqx_trie_nif:insert / delete),
%%   emqx_route events     -> the route bag   (emqx_trie_nif:route_write /
%%                            route_delete_object, which never touch the trie).
%% So the node-down cleanup (emqx_router_helper:cleanup_routes/1,
%% src/emqx_router_helper.erl:118-124, 156-160), which deletes route objects
%% and no trie node, leaves its stale filters in the engine's trie as it
%% leaves them in emqx_trie: match/1 keeps returning them and match_routes/1
%% finds no routes for them.  (tests/test_feed_replay.py replays such event
%% sequences through emqx_amd/feed.py, this module's mirror.)
%%
%% Deltas are applied at once to the engine's host trie; the upload to HBM is
%% batched every ?COMMIT_MS (the next match also commits implicitly, so a
%% publish never sees an older state than the last event handled here).
%% Visibility: the engine sees committed state only.  A match inside a mnesia
%% transaction does not see that transaction's own uncommitted trie writes,
%% as emqx_trie:match/1 does there (test/emqx_trie_SUITE.erl:60-68); the
%% production caller matches outside any transaction, under mnesia:ets/2
%% (src/emqx_router.erl:117), where the two agree.
-module(emqx_trie_gpu_feed).

-behaviour(gen_server).

-include_lib("emqx/include/emqx.hrl").

-export([start_link/0]).
-export([init/1, handle_call/3, handle_cast/2, handle_info/2, terminate/2, code_change/3]).

-define(TAB, emqx_trie_gpu).
-define(COMMIT_MS, 5).

start_link() ->
    gen_server:start_link({local, ?MODULE}, ?MODULE, [], []).

init([]) ->
    Devices = application:get_env(emqx, trie_gpu_devices, [0]),
    {ok, E} = emqx_trie_nif:open(Devices),
    _ = ets:new(?TAB, [named_table, public, set, {read_concurrency, true}]),
    true = ets:insert(?TAB, {engine, E}),
    %% subscribe first, snapshot second (see the header)
    {ok, _} = mnesia:subscribe({table, emqx_trie_node, detailed}),
    {ok, _} = mnesia:subscribe({table, emqx_route, detailed}),
    [ok = emqx_trie_nif:insert(E, T) || #trie_node{topic = T} <- ets:tab2list(emqx_trie_node),
                                        T =/= undefined],
    [ok = route_write(E, R) || R <- ets:tab2list(emqx_route)],
    {ok, _} = emqx_trie_nif:commit(E),
    {ok, #{engine => E, timer => undefined}}.

handle_call(_Req, _From, S) ->
    {reply, ignored, S}.

handle_cast(_Msg, S) ->
    {noreply, S}.

%% emqx_trie_node: a node whose topic is set is a filter (topic =:= node_id);
%% a write with topic undefined clears it (emqx_trie:delete/1 :94) or is an
%% intermediate node (add_path/1, delete_path/1): delete of a non-filter is a
%% no-op in the engine, as the trie's structure follows its filter set
handle_info({mnesia_table_event, {write, emqx_trie_node, #trie_node{topic = T}, _Old, _Tid}},
            S = #{engine := E}) when T =/= undefined ->
    ok = emqx_trie_nif:insert(E, T),
    {noreply, schedule_commit(S)};
handle_info({mnesia_table_event, {write, emqx_trie_node, #trie_node{node_id = N, topic = undefined}, _, _}},
            S = #{engine := E}) when is_binary(N) ->
    ok = emqx_trie_nif:delete(E, N),
    {noreply, schedule_commit(S)};
handle_info({mnesia_table_event, {delete, emqx_trie_node, {emqx_trie_node, N}, _Old, _Tid}},
            S = #{engine := E}) when is_binary(N) ->
    ok = emqx_trie_nif:delete(E, N),
    {noreply, schedule_commit(S)};
%% emqx_route (bag): one event per route object; the bag only
handle_info({mnesia_table_event, {write, emqx_route, #route{} = R, _Old, _Tid}}, S = #{engine := E}) ->
    ok = route_write(E, R),
    {noreply, schedule_commit(S)};
handle_info({mnesia_table_event, {delete_object, emqx_route, #route{topic = T, dest = D}, _Old, _Tid}},
            S = #{engine := E}) ->
    ok = emqx_trie_nif:route_delete_object(E, T, term_to_binary(D)),
    {noreply, schedule_commit(S)};
handle_info({mnesia_table_event, {delete, emqx_route, {emqx_route, T}, Old, _Tid}}, S = #{engine := E}) ->
    [ok = emqx_trie_nif:route_delete_object(E, T, term_to_binary(D)) || #route{dest = D} <- Old],
    {noreply, schedule_commit(S)};
handle_info({mnesia_table_event, _Other}, S) ->
    {noreply, S};
handle_info(commit, S = #{engine := E}) ->
    {ok, _Epoch} = emqx_trie_nif:commit(E),
    {noreply, S#{timer := undefined}};
handle_info(_Info, S) ->
    {noreply, S}.

terminate(_Reason, _S) ->
    ok.

code_change(_OldVsn, S, _Extra) ->
    {ok, S}.

%% a route and its dest's aggre/1 target: a node atom, or the $share group
%% of a {Group, Node} dest
route_write(E, #route{topic = T, dest = D}) ->
    DestBin = term_to_binary(D),
    ok = case D of
             {Group, _Node} -> emqx_trie_nif:dest_target(E, DestBin, group, Group);
             Node when is_atom(Node) -> emqx_trie_nif:dest_target(E, DestBin, node, atom_to_binary(Node, utf8))
         end,
    emqx_trie_nif:route_write(E, T, DestBin).

schedule_commit(S = #{timer := undefined}) ->
    S#{timer := erlang:send_after(?COMMIT_MS, self(), commit)};
schedule_commit(S) ->
    S.

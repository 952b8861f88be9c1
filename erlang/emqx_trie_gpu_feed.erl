%% emqx_trie_gpu_feed — keeps the GPU engine's image equal to the committed
%% mnesia state (SURVEY H4).  A child of emqx_sup next to emqx_router_sup
%% (src/emqx_sup.erl:57-88):
%%
%%   {emqx_trie_gpu_feed, {emqx_trie_gpu_feed, start_link, []},
%%    permanent, 5000, worker, [emqx_trie_gpu_feed]}
%%
%% At boot it opens the engine on the GPUs of app env {emqx, trie_gpu_devices}
%% (an integer or a list; default [0]), loads the current trie filters and
%% routes, and subscribes to the tables' detailed events.  Local transactions
%% (emqx_router add/del_trie_route, src/emqx_router.erl:226-260) and writes
%% replicated from other nodes (src/emqx_trie.erl:50-54) arrive the same way,
%% after commit, so an aborted transaction never reaches the image.  Deltas
%% are applied at once to the engine's host trie; the upload of dirty pages to
%% HBM is batched every ?COMMIT_MS (the next match also commits implicitly, so
%% a publish never sees an older state than the last event handled here).
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
    %% the committed state so far: filters of the trie, then the route bag
    [ok = emqx_trie_nif:insert(E, T) || #trie_node{topic = T} <- ets:tab2list(emqx_trie_node),
                                        T =/= undefined],
    [ok = add_route(E, R) || R <- ets:tab2list(emqx_route)],
    {ok, _} = emqx_trie_nif:commit(E),
    {ok, _} = mnesia:subscribe({table, emqx_trie_node, detailed}),
    {ok, _} = mnesia:subscribe({table, emqx_route, detailed}),
    {ok, #{engine => E, timer => undefined}}.

handle_call(_Req, _From, S) ->
    {reply, ignored, S}.

handle_cast(_Msg, S) ->
    {noreply, S}.

%% emqx_trie_node: a node whose topic is set is a filter (topic =:= node_id)
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
%% emqx_route (bag): one event per route object
handle_info({mnesia_table_event, {write, emqx_route, #route{} = R, _Old, _Tid}}, S = #{engine := E}) ->
    ok = add_route(E, R),
    {noreply, schedule_commit(S)};
handle_info({mnesia_table_event, {delete_object, emqx_route, #route{topic = T, dest = D}, _Old, _Tid}},
            S = #{engine := E}) ->
    ok = emqx_trie_nif:route_del(E, T, term_to_binary(D)),
    {noreply, schedule_commit(S)};
handle_info({mnesia_table_event, {delete, emqx_route, {emqx_route, T}, Old, _Tid}}, S = #{engine := E}) ->
    [ok = emqx_trie_nif:route_del(E, T, term_to_binary(D)) || #route{dest = D} <- Old],
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
add_route(E, #route{topic = T, dest = D}) ->
    DestBin = term_to_binary(D),
    ok = case D of
             {Group, _Node} -> emqx_trie_nif:dest_target(E, DestBin, group, Group);
             Node when is_atom(Node) -> emqx_trie_nif:dest_target(E, DestBin, node, atom_to_binary(Node, utf8))
         end,
    emqx_trie_nif:route_add(E, T, DestBin).

schedule_commit(S = #{timer := undefined}) ->
    S#{timer := erlang:send_after(?COMMIT_MS, self(), commit)};
schedule_commit(S) ->
    S.

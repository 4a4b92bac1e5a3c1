#!/usr/bin/env python3
"""Design aid (CPU only): how many 64-node tiles the tile-active multi-source BFS would
process on G100, for a given tile order, against the dense pull.

  python scripts/tile_sim.py [--n 100] [--order grow|rowmajor|block]

For each 32-source batch (cluster order) it computes every source's BFS levels, then per
level step L the tiles that must be processed (neighbour tiles of tiles holding a node on
level L for some source), and the per-level critical path when tile t is owned by wave
t % 8 (max over waves of owned active tiles). Prints totals in slot-steps.
"""
import argparse
import collections

import numpy as np


def grid(n):
    V = n * n
    adj = [[] for _ in range(V)]
    for r in range(n):
        for c in range(n):
            u = r * n + c
            if c + 1 < n:
                adj[u].append(u + 1)
                adj[u + 1].append(u)
            if r + 1 < n:
                adj[u].append(u + n)
                adj[u + n].append(u)
    return V, adj


def bfs(adj, srcs, V):
    lvl = np.full(V, -1, dtype=np.int64)
    q = collections.deque()
    for s in srcs:
        lvl[s] = 0
        q.append(s)
    while q:
        u = q.popleft()
        for v in adj[u]:
            if lvl[v] < 0:
                lvl[v] = lvl[u] + 1
                q.append(v)
    return lvl


def cluster_order(V, adj, k=32):
    taken = np.zeros(V, bool)
    order = []
    for s in range(V):
        if taken[s]:
            continue
        got = 0
        seen = {s}
        q = collections.deque([s])
        while q and got < k:
            u = q.popleft()
            if not taken[u]:
                taken[u] = True
                order.append(u)
                got += 1
            for v in adj[u]:
                if v not in seen:
                    seen.add(v)
                    q.append(v)
    return order


def tile_order_grow(V, adj, T=64):
    l0 = bfs(adj, [0], V)
    root = int(np.argmax(l0))
    lr = bfs(adj, [root], V)
    seeds = np.lexsort((np.arange(V), lr))
    taken = np.zeros(V, bool)
    order = []
    for s in seeds:
        if taken[s]:
            continue
        q = collections.deque([s])
        taken[s] = True
        order.append(s)
        while q and len(order) % T:
            u = q.popleft()
            for v in adj[u]:
                if not taken[v] and len(order) % T:
                    taken[v] = True
                    order.append(v)
                    q.append(v)
        # leftover queue nodes stay untaken
    return np.array(order)


def tile_order_block(n, T=64):
    b = 8
    order = []
    for br in range(0, n, b):
        for bc in range(0, n, b):
            for r in range(br, min(br + b, n)):
                for c in range(bc, min(bc + b, n)):
                    order.append(r * n + c)
    return np.array(order)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--order", default="grow")
    ap.add_argument("--batches", type=int, default=40)
    args = ap.parse_args()
    V, adj = grid(args.n)
    if args.order == "grow":
        tord = tile_order_grow(V, adj)
    elif args.order == "block":
        tord = tile_order_block(args.n)
    else:
        tord = np.arange(V)
    tinv = np.empty(V, np.int64)
    tinv[tord] = np.arange(V)
    tile = tinv // 64
    NT = int(tile.max()) + 1
    nbt = [set([t]) for t in range(NT)]
    for u in range(V):
        for v in adj[u]:
            nbt[tile[u]].add(tile[v])
    print("tiles", NT, "max neighbour tiles", max(len(s) for s in nbt))
    co = cluster_order(V, adj)
    nb = (V + 31) // 32
    pick = np.linspace(0, nb - 1, args.batches).astype(int)
    dense = crit = work = 0
    for b in pick:
        srcs = co[32 * b: 32 * b + 32]
        L = np.stack([bfs(adj, [s], V) for s in srcs])  # 32 x V
        depth = int(L.max())
        dense += (depth + 1) * 20
        for step in range(depth + 1):
            em = np.unique(tile[np.any(L == step, axis=0)])
            act = set()
            for t in em:
                act |= nbt[t]
            act = np.array(sorted(act))
            # done tiles: every node reached by every source at level <= step
            done = np.array([np.all(L[:, tord[64 * t: 64 * t + 64]] <= step) for t in act], bool) if act.size else act
            act = act[~done] if act.size else act
            work += act.size
            if act.size:
                crit += np.bincount(act % 8, minlength=8).max()
    nbx = len(pick)
    print(f"per batch: dense {dense / nbx:.0f} slot-steps/wave, tile-active crit {crit / nbx:.0f}, "
          f"mean active tiles/step {work / max(1, dense / 20):.1f}")


if __name__ == "__main__":
    main()

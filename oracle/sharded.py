"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the per-rank phases of the sharded train
(pypardis_amd/distributed.py, pd_train_begin / pd_train_end).  It is the
owner-rule merge of ``oracle.pipeline`` (which restates what
R:dbscan/dbscan.py:153-165 and R:dbscan/aggregator.py:9-73 intend) cut at
the device boundary:

* ``phase_a`` — one rank's neighbourhoods: per-neighbourhood sklearn DBSCAN
  (R:dbscan/dbscan.py:12-34), local clusters glued through points that are
  core in two of this rank's neighbourhoods, component key = smallest global
  id of its core points; exports (global id, key) for core points that also
  live on another rank.
* ``phase_b`` — after the global key map: owner points take the key of their
  component (core) or the smallest key among their core neighbours (border).

tests/test_distributed.py drives these through torch.distributed (gloo,
world size 2 and 3) and checks the assembled labels against sklearn.
"""
from __future__ import annotations

import numpy as np

from . import _UF, dbscan, neighbors


def phase_a(X, eps, min_samples, ebox, owner, gid, xr, metric="euclidean"):
    X = np.asarray(X)
    X64 = X.astype(np.float64)
    n = len(X)
    ebox = np.asarray(ebox, np.float64).reshape(-1, 2, X.shape[1])
    owner = np.asarray(owner, np.int64)
    gid = np.asarray(gid, np.int64)
    xr = np.asarray(xr).astype(bool)
    P = len(ebox)
    members, local, node_base = [], [], [0]
    for L in range(P):
        m = np.all(ebox[L, 0] <= X64, axis=1) & np.all(ebox[L, 1] >= X64, axis=1)
        mem = np.nonzero(m)[0]
        lab, core, _, ncl = dbscan(X[mem], eps, min_samples, metric)
        members.append(mem)
        local.append((lab, core))
        node_base.append(node_base[-1] + ncl)
    uf = _UF(node_base[-1])
    first_node = np.full(n, -1, np.int64)
    for L in range(P):
        lab, core = local[L]
        for i, c, is_core in zip(members[L], lab, core):
            if is_core:
                node = node_base[L] + int(c)
                if first_node[i] < 0:
                    first_node[i] = node
                else:
                    uf.union(first_node[i], node)
    nroot = np.array([uf.find(v) for v in range(node_base[-1])], np.int64)
    gmin = np.full(node_base[-1], np.iinfo(np.int64).max, np.int64)
    for L in range(P):
        lab, core = local[L]
        m = core.astype(bool)
        np.minimum.at(gmin, nroot[node_base[L] + lab[m]], gid[members[L][m]])
    ex = np.nonzero((first_node >= 0) & xr)[0]
    exports = (gid[ex], gmin[nroot[first_node[ex]]])
    state = dict(X=X, eps=eps, metric=metric, members=members, local=local,
                 node_base=node_base, nroot=nroot, gmin=gmin, owner=owner, gid=gid, n=n)
    return state, exports


def phase_b(state, keymap=None):
    """keys[n] (int64, -1 = noise / not owned here), core[n] (owned core)."""
    n = state["n"]
    X = state["X"]
    gmin = state["gmin"].copy()
    if keymap is not None:   # (ids ascending, their global keys)
        ids, keys = (np.asarray(a, np.int64) for a in keymap)
        if len(ids):
            pos = np.minimum(np.searchsorted(ids, gmin), len(ids) - 1)
            hit = ids[pos] == gmin
            gmin[hit] = keys[pos[hit]]
    nroot, node_base, owner = state["nroot"], state["node_base"], state["owner"]
    key = np.full(n, -1, np.int64)
    is_core = np.zeros(n, np.uint8)
    for L, mem in enumerate(state["members"]):
        lab, core = state["local"][L]
        own = owner[mem] == L
        if not np.any(own):
            continue
        pos = np.nonzero(own)[0]
        cm = core[pos].astype(bool)
        key[mem[pos[cm]]] = gmin[nroot[node_base[L] + lab[pos[cm]]]]
        is_core[mem[pos[cm]]] = 1
        border = pos[~cm]
        if len(border):
            off, nbr = neighbors(X[mem], state["eps"], state["metric"])
            for b in border:
                js = nbr[off[b]:off[b + 1]]
                js = js[core[js].astype(bool)]
                if len(js):
                    key[mem[b]] = gmin[nroot[node_base[L] + lab[js]]].min()
    return key, is_core


def merge(gid, key):
    """Union of the exported (id, key) pairs over the ids they name
    (pd_merge_exports): (ids ascending, global key of each = its component's
    smallest id)."""
    gid = np.asarray(gid, np.int64)
    key = np.asarray(key, np.int64)
    ids = np.unique(np.concatenate([gid, key]))
    uf = _UF(len(ids))
    for a, b in zip(np.searchsorted(ids, gid).tolist(), np.searchsorted(ids, key).tolist()):
        uf.union(int(a), int(b))
    return ids, ids[np.array([uf.find(v) for v in range(len(ids))], np.int64)]

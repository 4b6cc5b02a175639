"""Window sharding across GPUs (one process per GPU).

Windows are independent, so a batch is split into per-rank
shards with no exchange during compute.  The reference fans out per contig
(kt_for over contigs, blockjoin.c:4560), which balances poorly (chr1 vs
chr21); here whole windows are dealt by longest-processing-time-first on a
cost estimate (reads x calls, the greedy loop's work).  The only exchange is a
final gather of the per-window int8 decisions (and the tags of joined windows)
so that the host that writes VCF/GTF sees every decision, in original window
order -- which also preserves the reference's first-wins merge of read tags
(blockjoin.c:4414-4421, 4579-4595).
"""
from __future__ import annotations

import heapq

import numpy as np

from .abi import WindowBatch

__all__ = ["window_costs", "lpt_partition", "lpt_bound", "shard", "aln_window_costs", "shard_aln",
           "group_copies", "split_groups", "gather_decisions"]


def window_costs(batch: WindowBatch) -> np.ndarray:
    """LPT cost of each window, reads x calls: the greedy
    chain has about R iterations, each over terms proportional to the
    window's calls."""
    ro = batch.win_read_off.astype(np.int64)
    co = batch.read_call_off.astype(np.int64)
    reads = np.diff(ro)
    calls = co[ro[1:]] - co[ro[:-1]]
    return reads.astype(np.float64) * np.maximum(calls, 1).astype(np.float64)


def lpt_partition(costs: np.ndarray, n_parts: int):
    """Longest-processing-time-first: returns n_parts sorted index arrays."""
    order = np.argsort(-np.asarray(costs, dtype=np.float64), kind="stable")
    heap = [(0.0, p) for p in range(n_parts)]
    parts = [[] for _ in range(n_parts)]
    for w in order:
        load, p = heapq.heappop(heap)
        parts[p].append(int(w))
        heapq.heappush(heap, (load + float(costs[w]), p))
    return [np.array(sorted(p), dtype=np.int64) for p in parts]


def shard(batch: WindowBatch, rank: int, world: int):
    """(window indices, sub-batch) owned by `rank`."""
    parts = lpt_partition(window_costs(batch), world)
    idx = parts[rank]
    return idx, batch.select(idx)


def aln_window_costs(aln) -> np.ndarray:
    """Record-level cost of each window: its SEQ + MM bytes (K0's work)."""
    wo = aln.win_rec_off.astype(np.int64)
    per = (aln.l_qseq.astype(np.int64) + 1) // 2 + np.diff(aln.mm_off.astype(np.int64))
    cs = np.concatenate([[0], np.cumsum(per)])
    return (cs[wo[1:]] - cs[wo[:-1]]).astype(np.float64)


def shard_aln(aln, rank: int, world: int):
    """(window indices, record-level sub-batch) owned by `rank`."""
    parts = lpt_partition(aln_window_costs(aln), world)
    idx = parts[rank]
    return idx, aln.select(idx)


def lpt_bound(costs: np.ndarray, n_parts: int) -> float:
    """Graham's bound on the largest LPT load: (4/3 - 1/(3m)) x OPT, with
    OPT >= max(mean load, largest window)."""
    c = np.asarray(costs, np.float64)
    opt_lo = max(float(c.sum()) / n_parts, float(c.max()) if c.size else 0.0)
    return (4.0 / 3.0 - 1.0 / (3.0 * n_parts)) * opt_lo


def group_copies(share: np.ndarray, n_base: int):
    """Device batches of a rank's share of a job made of copies (one per
    contig) of `n_base` base windows: job window j is copy j // n_base of base
    window j % n_base.  Batch k takes the k-th copy of every base window the
    rank holds, in base-window order, so a rank that owns whole copies uploads
    each as the base batch itself.  Returns [(job windows, base windows)]."""
    share = np.sort(np.asarray(share, np.int64))
    base = share % n_base
    occ = np.zeros(share.shape[0], np.int64)
    seen = {}
    for i, b in enumerate(base.tolist()):
        occ[i] = seen.get(b, 0)
        seen[b] = occ[i] + 1
    groups = []
    for k in range(int(occ.max()) + 1 if share.size else 0):
        m = np.flatnonzero(occ == k)
        m = m[np.argsort(base[m], kind="stable")]
        groups.append((share[m], base[m]))
    return groups


def split_groups(groups, n_min: int, base_costs: np.ndarray):
    """At least n_min batches (one per context of the GPU): each group is
    dealt heaviest first, round-robin, into ceil(n_min / len(groups)) parts."""
    if not groups or len(groups) >= n_min:
        return groups
    k = -(-n_min // len(groups))
    out = []
    for jobw, basew in groups:
        order = np.argsort(-np.asarray(base_costs, np.float64)[basew], kind="stable")
        for s in range(k):
            sel = np.sort(order[s::k])
            if sel.size:
                out.append((jobw[sel], basew[sel]))
    return out


def gather_decisions(n_windows: int, idx: np.ndarray, decision: np.ndarray, group=None):
    """All-gather per-window decisions into original window order.

    With torch.distributed initialised the int8 decisions travel over the
    default process group (RCCL on GPUs, gloo on CPU); without it the local
    shard is returned in place."""
    full = np.full(n_windows, -1, np.int8)
    try:
        import torch
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError
    except Exception:
        full[idx] = decision
        return full
    world = dist.get_world_size(group)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    # pack (window index, decision) pairs; shards have different sizes -> pad
    n_local = torch.tensor([len(idx)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n_local, group=group)
    mx = int(max(int(s.item()) for s in sizes))
    buf = torch.full((mx, 2), -1, dtype=torch.int64, device=dev)
    if len(idx):
        buf[:len(idx), 0] = torch.from_numpy(np.asarray(idx, np.int64)).to(dev)
        buf[:len(idx), 1] = torch.from_numpy(np.asarray(decision, np.int64)).to(dev)
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    for o in outs:
        o = o.cpu().numpy()
        ok = o[:, 0] >= 0
        full[o[ok, 0]] = o[ok, 1].astype(np.int8)
    return full

"""Seeded synthetic BAM records for the record-level path (pf_aln_batch_t).

The window model is synth.py's (lognormal 30+-15 kb
reads, CpGs every ~100 bp, 70/20/10 % methylated/unmethylated/allele-specific
sites, 5 % no-calls, HP tags by truth haplotype and window orientation), one
level lower: every read is a BAM record with a reference sequence, a CIGAR
with indels and soft clips, a 4-bit SEQ with substitutions and an MM/ML pair
in the encodings basecallers emit, so the device loader (K0) sees what
htslib would hand the reference's load_reads_given_interval
(blockjoin.c:1043-1173):

* reference: random bases with CpGs only where planted (accidental CG broken);
* reads: indel events at `indel_rate` per base (1-3 bases), substitutions at
  `sub_rate`, leading/trailing soft clips on `clip_frac` of the reads;
* calls: every CpG of the read's SEQ (the C for forward reads, the G of the
  stored CG for reverse reads, i.e. the C of the original read), MM skip
  counts among all C's of the original read orientation, ML from the call's
  category band; `implicit_frac` of the reads also call a few non-CpG C's,
  which switches the reference to its implicit-canonical mode (852-858);
* MM layouts: "C+m?" alone, "C+h?;C+m?" (ML of h first), combined "C+hm?",
  "C+m." and a missing ML tag, mixed when `mm_mix` is set;
* `filt_frac` of the records fail one of the loader's filters (flags
  4/256/2048, MAPQ, de, length).

Everything is a pure function of (seed, window index).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

from .abi import HAPTAG_UNPHASED, AlnBatch
from .synth import _lognormal_params

_NT16 = np.array([1, 2, 4, 8], np.uint8)      # A C G T (internal codes 0..3)
A_, C_, G_, T_ = 0, 1, 2, 3


@dataclass
class AlnSpec:
    n_windows: int = 256
    coverage: float = 30.0
    gap: int = 50_000
    readback: int = 50_000
    mean_len: float = 30_000.0
    sd_len: float = 15_000.0
    min_len: int = 15_000
    max_len: int = 150_000
    cpg_rate: float = 0.01
    nocall_frac: float = 0.05
    untag_frac: float = 0.10
    seed: int = 1
    window_stride: int = 600_000
    base: int = 1_000_000
    gap_mix: bool = False
    indel_rate: float = 0.004
    sub_rate: float = 0.005
    clip_frac: float = 0.3
    clip_max: int = 400
    implicit_frac: float = 0.0
    filt_frac: float = 0.02
    mm_mix: bool = False       # mix MM/ML layouts (tests); else "C+h?;C+m?" (dorado 5mCG_5hmCG)
    len_scale: float = 1.0     # scales read lengths and min_len-sensitive sizes (small tests)
    het_snv_rate: float = 0.0  # > 0: het SNVs outside the gap, alt on one truth haplotype, and MD:Z per record
    windows_at: tuple = ()     # explicit (s, e) per window index instead of the strided layout
    orient_at: tuple = ()      # explicit cis (0) / trans (1) per window index
    skip_frac: float = 0.0     # windows whose left-block reads lost their HP tags (skipped by 1161-1163)
    nosite_frac: float = 0.0   # windows without allele- or unmethylated sites (no site qualifies, 4266)


def _qual_from_cat(rng, cat):
    q = np.empty(cat.shape[0], np.uint8)
    m = cat == 0
    q[m] = rng.integers(200, 256, m.sum())
    m = cat == 1
    q[m] = rng.integers(0, 96, m.sum())
    m = cat == 2
    q[m] = rng.integers(100, 156, m.sum())
    return q


def make_aln_window(spec: AlnSpec, w: int):
    rng = np.random.default_rng([spec.seed, w, 77])
    gap = spec.gap
    if spec.gap_mix:
        gap = int(np.exp(rng.uniform(np.log(5_000), np.log(500_000))))
    max_len = int(spec.max_len * spec.len_scale)
    stride = max(spec.window_stride, gap + 2 * spec.readback + 2 * max_len + 10_000)
    # windows are independent: the layout wraps so that every position stays
    # below the 2^29 limit of the call packing (a human chromosome is < 2^28)
    s = spec.base + (w % max(1, (400_000_000 - spec.base) // stride)) * stride
    e = s + gap
    if spec.windows_at:
        s, e = (int(x) for x in spec.windows_at[w])
    f_lo, f_hi = max(0, s - spec.readback), e + spec.readback
    span_lo, span_hi = f_lo - max_len, f_hi + max_len
    L = span_hi - span_lo + 16

    # reference with CpGs only where planted
    ref = rng.integers(0, 4, L).astype(np.uint8)
    cg = np.flatnonzero((ref[:-1] == C_) & (ref[1:] == G_))
    ref[cg + 1] = A_
    n_cpg = rng.poisson(spec.cpg_rate * L)
    cpg = np.unique(rng.integers(1, L - 3, size=n_cpg))
    cpg = cpg[np.concatenate([[True], np.diff(cpg) >= 2])]
    ref[cpg] = C_
    ref[cpg + 1] = G_
    cls = rng.random(cpg.shape[0])
    site_p = np.where(cls < 0.7, 0.95, 0.05)
    site_asm = cls >= 0.9
    site_hap = rng.integers(0, 2, cpg.shape[0])
    # window kinds of real runs (a separate stream: other windows are unchanged)
    kind_u = np.random.default_rng([spec.seed, w, 79]).random()
    skip_window = kind_u < spec.skip_frac
    if spec.skip_frac <= kind_u < spec.skip_frac + spec.nosite_frac:
        site_p[:] = 0.95
        site_asm[:] = False
    site_of = np.full(L, -1, np.int64)
    site_of[cpg] = np.arange(cpg.shape[0])
    snv = _plant_snvs(spec, w, ref, cpg, span_lo, s, e) if spec.het_snv_rate > 0 else None

    # reads (reference spans), tags as synth.py
    mu, sig = _lognormal_params(spec.mean_len * spec.len_scale, spec.sd_len * spec.len_scale)
    n_draw = int(spec.coverage * (span_hi - span_lo) / (spec.mean_len * spec.len_scale))
    starts = rng.integers(span_lo, f_hi, size=n_draw, dtype=np.int64)
    lens = np.clip(np.exp(rng.normal(mu, sig, n_draw)), spec.min_len * spec.len_scale, max_len).astype(np.int64)
    ends = starts + lens
    keep = (ends > f_lo) & (starts < f_hi) & (starts >= 0)
    starts, ends, lens = starts[keep], ends[keep], lens[keep]
    order = np.argsort(starts, kind="stable")
    starts, ends, lens = starts[order], ends[order], lens[order]
    n = starts.shape[0]
    truth = rng.integers(0, 2, n)
    orient = int(rng.integers(0, 2))
    if spec.orient_at:
        orient = int(spec.orient_at[w])
    hp = np.full(n, HAPTAG_UNPHASED, np.int64)
    tl = starts < s
    hp[tl] = truth[tl]
    only_right = (~tl) & (ends > e)
    hp[only_right] = truth[only_right] ^ orient
    hp[rng.random(n) < spec.untag_frac] = HAPTAG_UNPHASED
    if skip_window:
        hp[tl & (np.arange(n) % 4 != 0)] = HAPTAG_UNPHASED
    strand = (rng.random(n) < 0.5).astype(np.int64)
    out, flag, mapq, de = _build_reads(spec, rng, ref, starts - span_lo, lens, truth, strand,
                                       site_of, site_p, site_asm, site_hap, snv)
    res = dict(s=s, e=e, orient=orient, pos=starts, flag=flag, mapq=mapq, de=de, hp=hp, recs=out)
    if snv is not None:
        res["snv"] = dict(pos=snv["pos"] + span_lo, ref=snv["ref"], alt=snv["alt"], h_alt=snv["h_alt"])
    return res



def _build_reads(spec: AlnSpec, rng, ref: np.ndarray, rs0: np.ndarray, lens: np.ndarray, truth: np.ndarray,
                 strand: np.ndarray, site_of: np.ndarray, site_p: np.ndarray, site_asm: np.ndarray,
                 site_hap: np.ndarray, snv):
    """BAM records of reads at ref-relative starts rs0 with reference spans
    lens: CIGAR with indel events and soft clips, 4-bit SEQ (the reference,
    the read's het SNV alleles, substitutions), MD:Z when snv is given, and
    the MM/ML pair of the read's CpG calls; then flag / MAPQ / de with the
    filter failures.  -> (records, flag, mapq, de)."""
    n = rs0.shape[0]

    # indel events, non-overlapping, strictly inside each read
    n_ev = rng.poisson(spec.indel_rate * lens)
    n_ev = np.minimum(n_ev, np.maximum(lens // 8, 0))
    ev_read = np.repeat(np.arange(n), n_ev)
    ev_pos = rs0[ev_read] + 1 + (rng.random(ev_read.shape[0]) * (lens[ev_read] - 8)).astype(np.int64)
    ev_len = rng.integers(1, 4, ev_read.shape[0])
    ev_ins = rng.random(ev_read.shape[0]) < 0.5
    o = np.lexsort((ev_pos, ev_read))
    ev_read, ev_pos, ev_len, ev_ins = ev_read[o], ev_pos[o], ev_len[o], ev_ins[o]
    BIG = np.int64(1) << 40
    key = ev_read * BIG + ev_pos
    endk = key + np.where(ev_ins, 0, ev_len)
    prev_end = np.concatenate([[np.int64(-1)], np.maximum.accumulate(endk)[:-1]])
    ok = key > prev_end
    ev_read, ev_pos, ev_len, ev_ins = ev_read[ok], ev_pos[ok], ev_len[ok], ev_ins[ok]
    n_ev = np.bincount(ev_read, minlength=n)
    ev_first = np.concatenate([[0], np.cumsum(n_ev)])

    # cursor before each event: read start or previous event's end
    is_first = np.zeros(ev_read.shape[0], bool)
    is_first[ev_first[:-1][n_ev > 0]] = True
    prev_cur = np.empty(ev_read.shape[0], np.int64)
    if ev_read.shape[0]:
        prev_cur[1:] = ev_pos[:-1] + np.where(ev_ins[:-1], 0, ev_len[:-1])
        prev_cur[is_first] = rs0[ev_read[is_first]]
    m_before = ev_pos - prev_cur                           # >= 1 by construction
    last_cur = rs0.copy()
    has_ev = n_ev > 0
    li = ev_first[1:][has_ev] - 1
    last_cur[has_ev] = ev_pos[li] + np.where(ev_ins[li], 0, ev_len[li])
    m_last = rs0 + lens - last_cur

    # soft clips
    clip = rng.random(n) < spec.clip_frac
    c1 = np.where(clip & (rng.random(n) < 0.7), rng.integers(1, spec.clip_max, n), 0)
    c2 = np.where(clip & (rng.random(n) < 0.7), rng.integers(1, spec.clip_max, n), 0)

    # per read: ops  [S c1] (M_k, E_k)* M_last [S c2]
    recs = []
    ins_total = ev_len[ev_ins]
    for r in range(n):
        k0, k1 = ev_first[r], ev_first[r + 1]
        ne = k1 - k0
        core_len = np.empty(2 * ne + 1, np.int64)
        core_op = np.empty(2 * ne + 1, np.int64)
        core_len[0:2 * ne:2] = m_before[k0:k1]
        core_op[0:2 * ne:2] = 0
        core_len[1:2 * ne:2] = ev_len[k0:k1]
        core_op[1:2 * ne:2] = np.where(ev_ins[k0:k1], 1, 2)
        core_len[-1] = m_last[r]
        core_op[-1] = 0
        # SEQ: reference bases of M ops, random bases of I ops
        ref_cur = rs0[r] + np.concatenate([[0], np.cumsum(np.where(core_op == 1, 0, core_len))[:-1]])
        qlen = np.where(core_op == 2, 0, core_len)
        tot = int(qlen.sum())
        q0 = np.concatenate([[0], np.cumsum(qlen)[:-1]])
        idx = np.repeat(ref_cur - q0, qlen) + np.arange(tot)
        kind = np.repeat(core_op, qlen)
        bases = ref[np.where(kind == 0, idx, 0)]
        refpos = np.where(kind == 0, idx, -1)
        if snv is not None:                                   # het SNV alleles of the read's haplotype
            on = (kind == 0) & (snv["alt_of"][np.maximum(idx, 0)] >= 0)
            on &= snv["halt_of"][np.maximum(idx, 0)] == truth[r]
            bases[on] = snv["alt_of"][idx[on]]
        ins_m = kind == 1
        bases[ins_m] = rng.integers(0, 4, int(ins_m.sum()))
        sub = (rng.random(tot) < spec.sub_rate) & ~ins_m
        bases[sub] = (bases[sub] + rng.integers(1, 4, int(sub.sum()))) % 4
        if c1[r] or c2[r]:
            bases = np.concatenate([rng.integers(0, 4, c1[r]).astype(np.uint8), bases,
                                    rng.integers(0, 4, c2[r]).astype(np.uint8)])
            refpos = np.concatenate([np.full(c1[r], -1), refpos, np.full(c2[r], -1)])
        ops = []
        if c1[r]:
            ops.append((c1[r], 4))
        ops += list(zip(core_len.tolist(), core_op.tolist()))
        if c2[r]:
            ops.append((c2[r], 4))
        cigar = np.array([(l << 4) | op for l, op in ops], np.uint32)
        md = _md_string(bases[c1[r]:], ref, rs0[r], core_op, core_len) if snv is not None else None
        recs.append((bases, refpos, cigar, md))

    # calls per read
    out = []
    for r in range(n):
        bases, refpos, cigar, md_s = recs[r]
        lq = bases.shape[0]
        cgp = np.flatnonzero((bases[:-1] == C_) & (bases[1:] == G_))     # C of each CpG (stored)
        sid = site_of[np.maximum(refpos[cgp], 0)]
        sid[refpos[cgp] < 0] = -1
        p = np.full(cgp.shape[0], 0.5)
        on = sid >= 0
        p[on] = site_p[sid[on]]
        a = on & site_asm[np.maximum(sid, 0)]
        p[a] = np.where(site_hap[sid[a]] == truth[r], 0.95, 0.05)
        cat = np.where(rng.random(cgp.shape[0]) < p, 0, 1)
        cat[rng.random(cgp.shape[0]) < spec.nocall_frac] = 2
        called = cgp if strand[r] == 0 else cgp + 1                     # stored position of the called base
        if spec.implicit_frac and rng.random() < spec.implicit_frac:
            if strand[r] == 0:
                cand = np.flatnonzero((bases[:-1] == C_) & (bases[1:] != G_))
            else:
                cand = 1 + np.flatnonzero((bases[1:] == G_) & (bases[:-1] != C_))
            if cand.shape[0]:
                extra = rng.choice(cand, size=min(cand.shape[0], int(rng.integers(1, 4))), replace=False)
                called = np.concatenate([called, extra])
                cat = np.concatenate([cat, rng.integers(0, 3, extra.shape[0])])
                o = np.argsort(called, kind="stable")
                called, cat = called[o], cat[o]
        qual = _qual_from_cat(rng, cat)
        # MM skip counts in the original read orientation
        tb = C_ if strand[r] == 0 else G_
        allt = np.flatnonzero(bases == tb)
        rank = np.searchsorted(allt, called)
        if strand[r]:
            rank = allt.shape[0] - 1 - rank
            o = np.argsort(rank, kind="stable")
            rank, qual = rank[o], qual[o]
        deltas = np.diff(np.concatenate([[-1], rank])) - 1
        ds = ",".join(map(str, deltas.tolist()))
        style = int(rng.integers(0, 5)) if spec.mm_mix else 1
        nd = deltas.shape[0]
        if nd == 0:
            mm, ml = "", np.zeros(0, np.uint8)
        elif style == 0:
            mm, ml = f"C+m?,{ds};", qual
        elif style == 1:
            hq = rng.integers(0, 40, nd).astype(np.uint8)
            mm, ml = f"C+h?,{ds};C+m?,{ds};", np.concatenate([hq, qual])
        elif style == 2:
            hq = rng.integers(0, 40, nd).astype(np.uint8)
            mm, ml = f"C+hm?,{ds};", np.stack([hq, qual], 1).reshape(-1)
        elif style == 3:
            mm, ml = f"C+m.,{ds};", qual
        else:
            mm, ml = f"C+m?,{ds};", np.zeros(0, np.uint8)
        codes = _NT16[bases]
        if lq & 1:
            codes = np.concatenate([codes, np.zeros(1, np.uint8)])
        seq = (codes[0::2] << 4) | codes[1::2]
        out.append(dict(seq=seq, l_qseq=lq, cigar=cigar, mm=np.frombuffer(mm.encode(), np.uint8), ml=ml))
        if md_s is not None:
            out[-1]["md"] = md_s

    flag = (strand * 16).astype(np.uint16)
    mapq = np.full(n, 60, np.uint8)
    de = rng.uniform(0.01, 0.08, n).astype(np.float32)
    de[rng.random(n) < 0.1] = -1.0
    if spec.filt_frac:
        bad = np.flatnonzero(rng.random(n) < spec.filt_frac)
        kind = rng.integers(0, 5, bad.shape[0])
        flag[bad[kind == 0]] |= np.uint16(256)
        flag[bad[kind == 1]] |= np.uint16(2048)
        mapq[bad[kind == 2]] = 5
        de[bad[kind == 3]] = 0.2
        flag[bad[kind == 4]] |= np.uint16(4)
    return out, flag, mapq, de

def _plant_snvs(spec: AlnSpec, w: int, ref: np.ndarray, cpg: np.ndarray, span_lo: int, s: int, e: int):
    """Het SNVs for the -u path (a separate stream: the records of a spec
    without SNVs do not change).  Poisson at het_snv_rate outside the gap,
    plus one at each gap end (0-based s-1 and e-1: the last variant of the
    left phase block at POS s and the first of the right one at POS e, so
    that insert_vcf_line's gap is exactly [s, e]); never on a planted CpG.
    The ALT allele sits on truth haplotype h_alt."""
    rng = np.random.default_rng([spec.seed, w, 78])
    L = ref.shape[0]
    n = rng.poisson(spec.het_snv_rate * L)
    cand = np.unique(np.concatenate([rng.integers(2, L - 2, n), [s - 1 - span_lo, e - 1 - span_lo]]))
    g = cand + span_lo
    cand = cand[(g < s) | (g >= e - 1)]
    bad = np.zeros(L, bool)
    bad[cpg] = True
    bad[cpg + 1] = True
    keep = ~bad[cand] | np.isin(cand + span_lo, [s - 1, e - 1])   # the gap ends stay, CpG or not
    cand = cand[keep]
    refb = ref[cand].copy()
    alt = ((refb + rng.integers(1, 4, cand.shape[0])) % 4).astype(np.uint8)
    h_alt = rng.integers(0, 2, cand.shape[0]).astype(np.int64)
    alt_of = np.full(L, -1, np.int16)
    halt_of = np.full(L, -1, np.int16)
    alt_of[cand] = alt
    halt_of[cand] = h_alt
    return dict(pos=cand, ref=refb, alt=alt, h_alt=h_alt, alt_of=alt_of, halt_of=halt_of)


_ACGT = "ACGT"


def _md_string(core: np.ndarray, ref: np.ndarray, rs0: int, ops: np.ndarray, lens: np.ndarray) -> str:
    """SAM MD:Z of an alignment whose query (without the leading clip) is
    `core` against `ref` from ref index rs0, ops M/I/D only: the matched
    reference bases between consecutive events (a mismatching M base, a
    deletion), each event as its reference base or ^ + the deleted bases."""
    ops = np.asarray(ops, np.int64)
    lens = np.asarray(lens, np.int64)
    qlen = np.where(ops == 2, 0, lens)
    rlen = np.where(ops == 1, 0, lens)
    q0 = np.concatenate([[0], np.cumsum(qlen)[:-1]])
    r0 = int(rs0) + np.concatenate([[0], np.cumsum(rlen)[:-1]])
    m = ops == 0
    ml = lens[m]
    base = np.concatenate([[0], np.cumsum(ml)[:-1]])
    step = np.arange(int(ml.sum()), dtype=np.int64)
    qi = np.repeat(q0[m] - base, ml) + step
    ri = np.repeat(r0[m] - base, ml) + step
    mpos = ri[core[qi] != ref[ri]]
    d = ops == 2
    epos = np.concatenate([mpos, r0[d]])
    elen = np.concatenate([np.zeros(mpos.shape[0], np.int64), lens[d]])
    o = np.argsort(epos, kind="stable")
    parts, cur = [], int(rs0)
    for p, ln in zip(epos[o].tolist(), elen[o].tolist()):
        parts.append(str(p - cur))
        if ln == 0:
            parts.append(_ACGT[int(ref[p])])
            cur = p + 1
        else:
            parts.append("^" + "".join(_ACGT[int(b)] for b in ref[p:p + ln]))
            cur = p + ln
    parts.append(str(int(rs0) + int(rlen.sum()) - cur))
    return "".join(parts)


def _window_job(args):
    return make_aln_window(*args)


def window_cost_estimate(spec: AlnSpec, w: int) -> float:
    """The read bases of window w without building its reads: the same
    draws as make_aln_window up to the read spans (the RNG stream is
    replayed), the sum of the kept reads' lengths.  Proportional, up to
    clipping and indels, to the window's SEQ + MM bytes (shard.aln_window_costs),
    for dealing distinct windows before generating them."""
    rng = np.random.default_rng([spec.seed, w, 77])
    gap = spec.gap
    if spec.gap_mix:
        gap = int(np.exp(rng.uniform(np.log(5_000), np.log(500_000))))
    max_len = int(spec.max_len * spec.len_scale)
    stride = max(spec.window_stride, gap + 2 * spec.readback + 2 * max_len + 10_000)
    s = spec.base + (w % max(1, (400_000_000 - spec.base) // stride)) * stride
    e = s + gap
    if spec.windows_at:
        s, e = (int(x) for x in spec.windows_at[w])
    f_lo, f_hi = max(0, s - spec.readback), e + spec.readback
    span_lo, span_hi = f_lo - max_len, f_hi + max_len
    L = span_hi - span_lo + 16
    rng.integers(0, 4, L)
    n_cpg = rng.poisson(spec.cpg_rate * L)
    cpg = np.unique(rng.integers(1, L - 3, size=n_cpg))
    cpg = cpg[np.concatenate([[True], np.diff(cpg) >= 2])]
    rng.random(cpg.shape[0])
    rng.integers(0, 2, cpg.shape[0])
    if spec.het_snv_rate > 0:
        raise ValueError("window_cost_estimate: no -u windows")
    mu, sig = _lognormal_params(spec.mean_len * spec.len_scale, spec.sd_len * spec.len_scale)
    n_draw = int(spec.coverage * (span_hi - span_lo) / (spec.mean_len * spec.len_scale))
    starts = rng.integers(span_lo, f_hi, size=n_draw, dtype=np.int64)
    lens = np.clip(np.exp(rng.normal(mu, sig, n_draw)), spec.min_len * spec.len_scale, max_len).astype(np.int64)
    ends = starts + lens
    keep = (ends > f_lo) & (starts < f_hi) & (starts >= 0)
    return float(lens[keep].sum())


def _cost_job(args):
    return window_cost_estimate(*args)


def window_cost_estimates(jobs, workers: int = 16) -> np.ndarray:
    """window_cost_estimate over (spec, w) pairs, in worker processes."""
    jobs = list(jobs)
    if workers > 1 and len(jobs) >= 16:
        import multiprocessing as mp
        with mp.get_context("fork").Pool(workers) as pool:
            return np.array(pool.map(_cost_job, jobs, chunksize=16), np.float64)
    return np.array([window_cost_estimate(*j) for j in jobs], np.float64)


def make_aln_batch(spec: AlnSpec, windows=None, workers: int = 0, jobs=None) -> AlnBatch:
    """workers: processes generating windows in parallel (0: up to 16 when
    there are many windows; every window is a pure function of its index,
    so the result does not depend on it).  jobs: (spec, window) pairs
    instead of `windows` of `spec` (windows of several seeds in one batch)."""
    if jobs is None:
        if windows is None:
            windows = range(spec.n_windows)
        jobs = [(spec, w) for w in windows]
    jobs = list(jobs)
    if workers == 0:
        env = os.environ.get("PF_SYNTH_WORKERS")
        workers = int(env) if env else (min(16, os.cpu_count() or 1) if len(jobs) >= 16 else 1)
    if workers > 1:
        import multiprocessing as mp
        with mp.get_context("fork").Pool(workers) as pool:
            parts = pool.map(_window_job, jobs, chunksize=1)
    else:
        parts = [make_aln_window(*j) for j in jobs]
    recs = [r for p in parts for r in p["recs"]]

    def off(key, f=lambda x: x.shape[0]):
        return np.concatenate([[0], np.cumsum([f(r[key]) for r in recs])]).astype(np.uint64)

    def cat(key, dt):
        return np.concatenate([r[key] for r in recs]).astype(dt) if recs else np.zeros(0, dt)

    rc = np.array([len(p["recs"]) for p in parts], np.int64)
    b = AlnBatch(
        win_start=np.array([p["s"] for p in parts], np.uint32),
        win_end=np.array([p["e"] for p in parts], np.uint32),
        win_rec_off=np.concatenate([[0], np.cumsum(rc)]).astype(np.uint32),
        flag=np.concatenate([p["flag"] for p in parts]) if parts else np.zeros(0, np.uint16),
        mapq=np.concatenate([p["mapq"] for p in parts]) if parts else np.zeros(0, np.uint8),
        pos=np.concatenate([p["pos"] for p in parts]) if parts else np.zeros(0, np.uint32),
        l_qseq=np.array([r["l_qseq"] for r in recs], np.uint32),
        de=np.concatenate([p["de"] for p in parts]) if parts else np.zeros(0, np.float32),
        hp=np.concatenate([p["hp"] for p in parts]) if parts else np.zeros(0, np.uint8),
        cigar_off=off("cigar"), cigar=cat("cigar", np.uint32),
        seq_off=off("seq"), seq=cat("seq", np.uint8),
        mm_off=off("mm"), mm=cat("mm", np.uint8),
        ml_off=off("ml"), ml=cat("ml", np.uint8),
    )
    b.meta["orient"] = np.array([p["orient"] for p in parts], np.int8)
    b.meta["spec"] = spec
    if spec.het_snv_rate > 0:
        b.meta["md"] = [r["md"] for r in recs]
        b.meta["snv"] = [p["snv"] for p in parts]
    return b


_SAVE_FIELDS = ("win_start", "win_end", "win_rec_off", "flag", "mapq", "pos", "l_qseq", "de", "hp",
                "cigar_off", "cigar", "seq_off", "seq", "mm_off", "mm", "ml_off", "ml")


def save_aln(path: str, aln: AlnBatch) -> None:
    """Write a record-level batch as a plain .npz (no pickled objects)."""
    np.savez(path, orient=aln.meta.get("orient", np.zeros(0, np.int8)),
             **{k: getattr(aln, k) for k in _SAVE_FIELDS})


def load_aln(path: str) -> AlnBatch:
    with np.load(path, allow_pickle=False) as z:
        b = AlnBatch(**{k: z[k] for k in _SAVE_FIELDS})
        b.meta["orient"] = z["orient"]
    return b

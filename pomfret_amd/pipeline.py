"""`pomfret methphase` / `pomfret report` end to end: a thin binding of the C
pipeline driver (pomfret_amd/csrc/pf_pipeline.c, the pf_methphase_main /
pf_mp_* entry points of include/pomfret_amd.h).  The host side is C:

    f3  pf_vcf_gaps                 phase-block gaps of the phased VCF
                                    (load_intervals_from_file + merge_close_intervals,
                                    blockjoin.c:4442-4523)
    -u  pf_haptag_reads per contig  K4 pre-pass, qname first-wins per contig,
                                    merged in contig order (1841-1898, 2069-2080)
    f1  pf_bam_fetch_windows        each job's records (1053-1076), overlapped
                                    with the previous job's kernels
    GPU pf_batch_upload_aln + pf_methphase_run: K0 loader, K12, K3 (the kt_for
                                    worker, 4340-4426)
    a1  first-wins qname -> hp of joined windows, in (contig, window) order
                                    (4408-4423, 4572-4595), a C table (pf_tags_t)
    f2  pf_phase_blocks, pf_write_gtf / _tsv / _vcf + pf_rescue_dropped
                                    (lift_decisions ... output_modify_vcf, 4685-4717)

`methphase_files` runs everything in this process (one host thread per GPU
it drives).  `methphase_files_dist` is the one-process-per-GPU form: every
rank builds the same plan, runs the jobs its static LPT shard owns, and the
job results (per-window decisions + the joined windows' qname/tag lists)
are gathered over torch.distributed to rank 0, which merges them in window
order and writes the outputs -- the merged tables equal the single-process
ones exactly.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Dict, List, Optional

import numpy as np

from ._lib import (INTERVALS_GTF, INTERVALS_TSV, INTERVALS_VCF, PomfretError, _blocks_contigs, _check,  # noqa: F401
                   _gaps_contigs, _PfBlocks, _PfGaps, lib)
from .abi import Config, LoadConfig, PfCfg, PfLoadCfg

MODE_METHPHASE, MODE_REPORT = 0, 1
JOB_WINDOWS, JOB_HAPTAG = 0, 1


class PfMethphaseOpts(C.Structure):
    _fields_ = [("mode", C.c_int32), ("bam_path", C.c_char_p), ("vcf_path", C.c_char_p),
                ("out_prefix", C.c_char_p), ("cov_for_selection", C.c_int32), ("cov_for_runtime", C.c_int32),
                ("n_cand", C.c_int32), ("cov", C.c_int32), ("k", C.c_int32), ("k_span", C.c_int32),
                ("load", PfLoadCfg), ("untagged", C.c_int32), ("write_tsv", C.c_int32), ("write_bam", C.c_int32),
                ("chunk_size", C.c_int32), ("chunk_stride", C.c_int32), ("threads", C.c_int32),
                ("n_devices", C.c_int32), ("devices", C.c_void_p), ("ctxs", C.c_void_p), ("n_ctxs", C.c_int32),
                ("rank", C.c_int32), ("world", C.c_int32), ("job_windows", C.c_uint32), ("verbose", C.c_int32),
                ("host_fetch", C.c_int32), ("interval_path", C.c_char_p), ("interval_format", C.c_int32),
                ("write_input_tagging", C.c_int32), ("bam_threads", C.c_int32)]


class PfQnameTagsC(C.Structure):
    _fields_ = [("n", C.c_uint32), ("off", C.c_void_p), ("names", C.c_void_p), ("hp", C.c_void_p)]


class PfMpJobInfo(C.Structure):
    _fields_ = [("contig", C.c_uint32), ("contig_name", C.c_char_p), ("w0", C.c_uint32), ("w1", C.c_uint32),
                ("rank", C.c_int32), ("lpt_pos", C.c_uint32), ("cost", C.c_double), ("done", C.c_int32),
                ("cfg", PfCfg)]


class PfMpStats(C.Structure):
    _fields_ = [("s_plan", C.c_double), ("s_estimate", C.c_double), ("s_haptag", C.c_double),
                ("s_windows", C.c_double), ("s_finish", C.c_double), ("fetch_ms", (C.c_double * 7) * 2),
                ("comp_bytes", C.c_uint64 * 2), ("inflated_bytes", C.c_uint64 * 2), ("run_ms", C.c_double * 2),
                ("n_fetch", C.c_uint64 * 2), ("arena_hits", C.c_uint64), ("arena_misses", C.c_uint64),
                ("reread_bytes", C.c_uint64), ("steals", C.c_uint64)]


class PfMpJobResult(C.Structure):
    _fields_ = [("n_windows", C.c_uint32), ("decision", C.c_void_p), ("tag_off", C.c_void_p),
                ("tags", PfQnameTagsC), ("n_limit", C.c_uint32)]


_bound = False


def _bind():
    global _bound
    L = lib()
    if _bound:
        return L
    vp, u32, i32 = C.c_void_p, C.c_uint32, C.c_int
    L.pf_methphase_main.argtypes = [C.POINTER(PfMethphaseOpts), C.POINTER(vp)]
    L.pf_mp_plan.argtypes = [C.POINTER(PfMethphaseOpts), C.POINTER(vp)]
    L.pf_mp_free.argtypes = [vp]
    L.pf_mp_n_jobs.argtypes = [vp, i32]
    L.pf_mp_n_jobs.restype = u32
    L.pf_mp_job_info.argtypes = [vp, i32, u32, C.POINTER(PfMpJobInfo)]
    L.pf_mp_windows.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), C.POINTER(u32)]
    L.pf_mp_run_mine.argtypes = [vp, C.POINTER(PfMethphaseOpts), i32]
    L.pf_mp_run_job.argtypes = [vp, vp, u32]
    L.pf_mp_run_haptag_job.argtypes = [vp, vp, u32]
    L.pf_mp_merge_raw.argtypes = [vp]
    L.pf_mp_get_job_result.argtypes = [vp, i32, u32, C.POINTER(PfMpJobResult)]
    L.pf_mp_set_job_result.argtypes = [vp, i32, u32, C.POINTER(PfMpJobResult)]
    L.pf_mp_finish.argtypes = [vp]
    L.pf_mp_decisions.argtypes = [vp, C.POINTER(vp), C.POINTER(u32), C.POINTER(u32)]
    L.pf_mp_gaps.argtypes = [vp]
    L.pf_mp_gaps.restype = C.POINTER(_PfGaps)
    L.pf_mp_blocks.argtypes = [vp]
    L.pf_mp_blocks.restype = C.POINTER(_PfBlocks)
    L.pf_mp_qname_hp.argtypes = [vp]
    L.pf_mp_qname_hp.restype = vp
    L.pf_mp_raw_hp.argtypes = [vp]
    L.pf_mp_raw_hp.restype = vp
    L.pf_mp_report_counts.argtypes = [vp, C.POINTER(C.c_double)]
    L.pf_mp_stats.argtypes = [vp, C.POINTER(PfMpStats)]
    L.pf_tags_new.restype = vp
    L.pf_tags_free.argtypes = [vp]
    L.pf_tags_size.argtypes = [vp]
    L.pf_tags_size.restype = C.c_uint64
    L.pf_tags_put_first.argtypes = [vp, u32, vp, vp, vp]
    L.pf_tags_put_first.restype = C.c_int64
    L.pf_tags_get.argtypes = [vp, u32, vp, vp, C.c_uint8, vp]
    L.pf_tags_get.restype = C.c_int64
    L.pf_tags_view.argtypes = [vp, C.POINTER(PfQnameTagsC)]
    _bound = True
    return L


def _arr(ptr, n, dt) -> np.ndarray:
    n = int(n)
    if n == 0 or not ptr:
        return np.zeros(0, dt)
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dt))), (n,)).copy()


def _names_list(off: np.ndarray, names: np.ndarray) -> List[str]:
    b = names.tobytes()
    return [b[off[i]:off[i + 1]].decode("ascii", "replace") for i in range(len(off) - 1)]


def _pack_names(names: List[str]):
    enc = [q.encode() for q in names]
    off = np.zeros(len(enc) + 1, np.uint64)
    if enc:
        off[1:] = np.cumsum([len(q) for q in enc])
    buf = np.frombuffer(b"".join(enc) or b"\0", np.uint8).copy()
    return off, buf


def tags_dict(t) -> Dict[str, int]:
    """A pf_tags_t as {qname: hp} in insertion order."""
    L = _bind()
    if not t:
        return {}
    v = PfQnameTagsC()
    _check(L.pf_tags_view(t, C.byref(v)), "pf_tags_view")
    off = _arr(v.off, v.n + 1, np.uint64)
    names = _arr(v.names, off[-1] if v.n else 0, np.uint8)
    hp = _arr(v.hp, v.n, np.uint8)
    return dict(zip(_names_list(off, names), hp.tolist()))


class Tags:
    """Owned pf_tags_t (first-wins qname -> hp)."""

    def __init__(self):
        self.h = _bind().pf_tags_new()
        if not self.h:
            raise PomfretError("pf_tags_new")

    def put_first(self, names: List[str], hp) -> int:
        off, buf = _pack_names(names)
        hp = np.ascontiguousarray(np.asarray(hp, np.uint8) if len(names) else np.zeros(1, np.uint8))
        r = lib().pf_tags_put_first(self.h, len(names), off.ctypes.data, buf.ctypes.data, hp.ctypes.data)
        if r < 0:
            _check(int(r), "pf_tags_put_first")
        return int(r)

    def get(self, names: List[str], default: int = 254) -> np.ndarray:
        off, buf = _pack_names(names)
        out = np.zeros(max(len(names), 1), np.uint8)
        r = lib().pf_tags_get(self.h, len(names), off.ctypes.data, buf.ctypes.data, default, out.ctypes.data)
        if r < 0:
            _check(int(r), "pf_tags_get")
        return out[:len(names)]

    def __len__(self):
        return int(lib().pf_tags_size(self.h))

    def to_dict(self) -> Dict[str, int]:
        return tags_dict(self.h)

    def close(self):
        if self.h:
            lib().pf_tags_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def make_opts(bam_path: str, vcf_path: str, out_prefix: Optional[str], cfg: Optional[Config],
              lcfg: Optional[LoadConfig] = None, mode: int = MODE_METHPHASE, untagged: bool = False,
              tsv: bool = False, threads: int = 8, n_devices: int = 0, ctxs=None, rank: int = 0, world: int = 1,
              job_windows: int = 0, cov: int = 0, chunk_size: int = 50_000, chunk_stride: int = 1_000_000,
              verbose: int = 0, host_fetch: bool = False, intervals=None, write_input_tagging: bool = False):
    """pf_methphase_opts_t from Python values.  cfg None: per-contig
    parameters from the BAM's coverage estimate (runs without -c).
    intervals: (path, INTERVALS_GTF | INTERVALS_TSV), the --gtf / --tsv phase
    blocks (vcf_path may then be None unless untagged)."""
    lcfg = lcfg or LoadConfig()
    o = PfMethphaseOpts()
    o.mode = mode
    o.bam_path = bam_path.encode()
    o.vcf_path = vcf_path.encode() if vcf_path else None
    if intervals is not None:
        o.interval_path = intervals[0].encode()
        o.interval_format = int(intervals[1])
    o.write_input_tagging = int(bool(write_input_tagging))
    o.out_prefix = out_prefix.encode() if out_prefix else None
    if cfg is not None:
        o.cov_for_selection, o.cov_for_runtime, o.n_cand = cfg.cov_for_selection, cfg.cov_for_runtime, cfg.n_cand
        o.k, o.k_span = cfg.k, cfg.k_span
    else:
        o.cov_for_selection, o.cov_for_runtime, o.n_cand, o.k, o.k_span = -1, 0, 15, 3, 5000
    o.cov = int(cov)
    o.load = lcfg.to_c()
    o.untagged = int(bool(untagged))
    o.write_tsv = int(bool(tsv))
    o.chunk_size, o.chunk_stride = int(chunk_size), int(chunk_stride)
    o.threads = int(threads)
    o.n_devices = int(n_devices)
    keep = None
    if ctxs:
        keep = (C.c_void_p * len(ctxs))(*[c.handle for c in ctxs])
        o.ctxs = C.cast(keep, C.c_void_p)
        o.n_ctxs = len(ctxs)
    o.rank, o.world = int(rank), int(world)
    o.job_windows = int(job_windows)
    o.verbose = int(verbose)
    o.host_fetch = int(bool(host_fetch))
    o._keep = keep
    return o


class Plan:
    """A pf_mp_plan_t: the deterministic job list of one run and its results."""

    def __init__(self, opts: PfMethphaseOpts, handle=None):
        L = _bind()
        self.opts = opts
        if handle is None:
            h = C.c_void_p()
            _check(L.pf_mp_plan(C.byref(opts), C.byref(h)), "pf_mp_plan")
            handle = h
        self.h = handle

    def n_jobs(self, kind: int = JOB_WINDOWS) -> int:
        return int(lib().pf_mp_n_jobs(self.h, kind))

    def job_info(self, kind: int, j: int) -> dict:
        i = PfMpJobInfo()
        _check(lib().pf_mp_job_info(self.h, kind, j, C.byref(i)), "pf_mp_job_info")
        c = i.cfg
        return dict(contig=int(i.contig), contig_name=i.contig_name.decode(), w0=int(i.w0), w1=int(i.w1),
                    rank=int(i.rank), lpt_pos=int(i.lpt_pos), cost=float(i.cost), done=bool(i.done),
                    cfg=Config(k=c.k, k_span=c.k_span, cov_for_selection=c.cov_for_selection,
                               cov_for_runtime=c.cov_for_runtime, n_cand=c.n_cand))

    def windows(self):
        ws, we, co, n = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_uint32()
        _check(lib().pf_mp_windows(self.h, C.byref(ws), C.byref(we), C.byref(co), C.byref(n)), "pf_mp_windows")
        nc = int(lib().pf_mp_gaps(self.h).contents.n_contigs)
        return _arr(ws, n.value, np.uint32), _arr(we, n.value, np.uint32), _arr(co, nc + 1, np.uint64)

    def run_mine(self, kind: int, n_devices: int = 0, ctxs=None):
        o = make_opts("", "", None, None, threads=self.opts.threads, n_devices=n_devices, ctxs=ctxs,
                      rank=self.opts.rank, world=self.opts.world)
        _check(lib().pf_mp_run_mine(self.h, C.byref(o), kind), "pf_mp_run_mine")

    def merge_raw(self):
        _check(lib().pf_mp_merge_raw(self.h), "pf_mp_merge_raw")

    def get_result(self, kind: int, j: int) -> dict:
        r = PfMpJobResult()
        _check(lib().pf_mp_get_job_result(self.h, kind, j, C.byref(r)), "pf_mp_get_job_result")
        n, t = int(r.n_windows), r.tags
        off = _arr(t.off, t.n + 1, np.uint64)
        return dict(decision=_arr(r.decision, n, np.int8), tag_off=_arr(r.tag_off, n + 1, np.uint64),
                    off=off, names=_arr(t.names, off[-1] if t.n else 0, np.uint8), hp=_arr(t.hp, t.n, np.uint8),
                    n_limit=int(r.n_limit))

    def set_result(self, kind: int, j: int, res: dict):
        dec = np.ascontiguousarray(res["decision"], np.int8)
        n = dec.shape[0]
        to = np.ascontiguousarray(res.get("tag_off", np.zeros(n + 1, np.uint64)), np.uint64)
        off = np.ascontiguousarray(res["off"], np.uint64)
        names = np.ascontiguousarray(res["names"] if len(res["names"]) else np.zeros(1, np.uint8), np.uint8)
        hp = np.ascontiguousarray(res["hp"] if len(res["hp"]) else np.zeros(1, np.uint8), np.uint8)
        decp = np.ascontiguousarray(dec if n else np.zeros(1, np.int8))
        r = PfMpJobResult(n, decp.ctypes.data, to.ctypes.data,
                          PfQnameTagsC(len(off) - 1, off.ctypes.data, names.ctypes.data, hp.ctypes.data),
                          int(res.get("n_limit", 0)))
        _check(lib().pf_mp_set_job_result(self.h, kind, j, C.byref(r)), "pf_mp_set_job_result")

    def finish(self):
        _check(lib().pf_mp_finish(self.h), "pf_mp_finish")

    def decisions(self) -> np.ndarray:
        d, n, nl = C.c_void_p(), C.c_uint32(), C.c_uint32()
        _check(lib().pf_mp_decisions(self.h, C.byref(d), C.byref(n), C.byref(nl)), "pf_mp_decisions")
        self.n_limit = int(nl.value)
        return _arr(d, n.value, np.int8)

    def qname_hp(self) -> Dict[str, int]:
        return tags_dict(lib().pf_mp_qname_hp(self.h))

    def raw_hp(self) -> Dict[str, int]:
        return tags_dict(lib().pf_mp_raw_hp(self.h))

    def contigs(self):
        return _blocks_contigs(lib().pf_mp_blocks(self.h))

    def gaps(self):
        return _gaps_contigs(lib().pf_mp_gaps(self.h))

    def report_counts(self):
        c = (C.c_double * 3)()
        _check(lib().pf_mp_report_counts(self.h, c), "pf_mp_report_counts")
        return dict(correct=int(c[0]), switch=int(c[1]), fail=int(c[2]))

    def stats(self) -> Dict:
        """Wall seconds per phase and the device-fetch sums of the run
        (pf_mp_stats; a measurement hook)."""
        st = PfMpStats()
        _check(lib().pf_mp_stats(self.h, C.byref(st)), "pf_mp_stats")
        names = ("read", "inflate", "chain", "decode", "select", "build", "total")
        out = {k: round(getattr(st, k), 4) for k in ("s_plan", "s_estimate", "s_haptag", "s_windows", "s_finish")}
        out.update({k: int(getattr(st, k)) for k in ("arena_hits", "arena_misses", "reread_bytes", "steals")})
        for i, kind in enumerate(("windows", "haptag")):
            out[kind] = dict({f"{n}_ms": round(st.fetch_ms[i][j], 2) for j, n in enumerate(names)},
                             comp_bytes=int(st.comp_bytes[i]), inflated_bytes=int(st.inflated_bytes[i]),
                             run_ms=round(st.run_ms[i], 2), n_fetch=int(st.n_fetch[i]))
        return out

    def close(self):
        if self.h:
            lib().pf_mp_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _result(plan: Plan, mode: int) -> Dict:
    dec = plan.decisions()
    if mode == MODE_REPORT:
        return dict(decision=dec, counts=plan.report_counts(), n_limit=plan.n_limit)
    return dict(decision=dec, contigs=plan.contigs(), qname_hp=plan.qname_hp(), raw_hp=plan.raw_hp(),
                n_limit=plan.n_limit, stats=plan.stats())


def methphase_files(bam_path: str, vcf_path: str, out_prefix: Optional[str], cfg: Optional[Config],
                    lcfg: Optional[LoadConfig] = None, device: int = 0, threads: int = 8, ctx=None,
                    untagged: bool = False, tsv: bool = False, n_devices: int = 1, job_windows: int = 0,
                    host_fetch: bool = False, ctxs=None, intervals=None,
                    write_input_tagging: bool = False) -> Dict:
    """`pomfret methphase` over every gap of vcf_path with the reads of
    bam_path, in this process (pf_methphase_main).  Writes out_prefix +
    .mp.gtf / .mp.vcf (and .mp.tsv with tsv=True, the reference's
    --output-tsv) unless out_prefix is None.  cfg None: no -c, per-contig
    parameters from the coverage estimate (4358-4390).  ctx: drive that
    context; ctxs: drive those contexts, one host thread each, over one job
    queue (two contexts of one device exercise the multi-GPU dispatcher);
    else n_devices GPUs from `device` on (0: all visible).
    Returns dict(decision=int8[n_gaps], contigs=[...], qname_hp={qname: hp},
    raw_hp={qname: hp} (the -u table), n_limit).  intervals=(path,
    INTERVALS_GTF | INTERVALS_TSV): the --gtf / --tsv phase blocks instead of
    the VCF's (vcf_path None: no VCF written); write_input_tagging: -U."""
    L = _bind()
    devs = None
    if ctx is not None:
        ctxs = [ctx]
    if not ctxs and device and n_devices >= 1:
        devs = (C.c_int32 * n_devices)(*range(device, device + n_devices))
    o = make_opts(bam_path, vcf_path, out_prefix, cfg, lcfg, untagged=untagged, tsv=tsv, threads=threads,
                  n_devices=0 if ctxs else n_devices, ctxs=ctxs or None,
                  job_windows=job_windows, host_fetch=host_fetch, intervals=intervals,
                  write_input_tagging=write_input_tagging)
    if devs is not None:
        o.devices = C.cast(devs, C.c_void_p)
    h = C.c_void_p()
    _check(L.pf_methphase_main(C.byref(o), C.byref(h)), "pf_methphase_main")
    plan = Plan(o, handle=h)
    try:
        return _result(plan, MODE_METHPHASE)
    finally:
        plan.close()


def report_files(bam_path: str, vcf_path: str, out_prefix: Optional[str], cov: int = 0,
                 chunk_size: int = 50_000, chunk_stride: int = 1_000_000, lcfg: Optional[LoadConfig] = None,
                 untagged: bool = False, threads: int = 8, ctx=None, n_devices: int = 1, k: int = 3,
                 k_span: int = 5000, host_fetch: bool = False, ctxs=None) -> Dict:
    """`pomfret report` (main_methreport, 4901-5089): chunk windows inside the
    phased blocks, one methphase decision each; writes
    {out_prefix}.report.tsv and the running totals to stdout.  cov: -c
    (0: the per-contig estimate).  Returns dict(decision, counts)."""
    L = _bind()
    if ctx is not None:
        ctxs = [ctx]
    o = make_opts(bam_path, vcf_path, out_prefix, Config(k=k, k_span=k_span), lcfg, mode=MODE_REPORT,
                  untagged=untagged, threads=threads, n_devices=0 if ctxs else n_devices,
                  ctxs=ctxs or None, cov=cov, chunk_size=chunk_size, chunk_stride=chunk_stride,
                  host_fetch=host_fetch)
    h = C.c_void_p()
    _check(L.pf_methphase_main(C.byref(o), C.byref(h)), "pf_methphase_main")
    plan = Plan(o, handle=h)
    try:
        return _result(plan, MODE_REPORT)
    finally:
        plan.close()


def methphase_files_dist(bam_path: str, vcf_path: str, out_prefix: Optional[str], cfg: Optional[Config],
                         lcfg: Optional[LoadConfig] = None, untagged: bool = False, tsv: bool = False,
                         threads: int = 8, ctx=None, group=None, job_windows: int = 0, mode: int = MODE_METHPHASE,
                         cov: int = 0, chunk_size: int = 50_000, chunk_stride: int = 1_000_000,
                         runner: Optional[Callable] = None, writer: int = 0, host_fetch: bool = False,
                         intervals=None, write_input_tagging: bool = False) -> Dict:
    """One process per GPU (torch.distributed initialised; RCCL on GPUs,
    gloo on CPU).  Every rank plans the same jobs and runs the ones its
    static LPT shard owns on `ctx` (or its LOCAL_RANK device); -u tables are
    all-gathered so every rank loads with the merged table; window-job
    results are gathered to `writer`, which merges them in (contig, window)
    order, writes the outputs and broadcasts the decisions.
    `runner(plan, kind, j) -> result dict` replaces the device for a job
    (the CPU tests plug the oracle in here)."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    o = make_opts(bam_path, vcf_path, out_prefix if rank == writer else None, cfg, lcfg, mode=mode,
                  untagged=untagged, tsv=tsv, threads=threads, rank=rank, world=world, job_windows=job_windows,
                  cov=cov, chunk_size=chunk_size, chunk_stride=chunk_stride, host_fetch=host_fetch,
                  intervals=intervals, write_input_tagging=write_input_tagging)
    plan = Plan(o)
    try:
        def run(kind):
            mine = [j for j in range(plan.n_jobs(kind)) if plan.job_info(kind, j)["rank"] == rank]
            if runner is not None:
                for j in mine:
                    plan.set_result(kind, j, runner(plan, kind, j))
            elif mine:
                if ctx is None:
                    import os
                    from ._lib import Context
                    run.ctx = getattr(run, "ctx", None) or Context(int(os.environ.get("LOCAL_RANK", "0")))
                    plan.run_mine(kind, ctxs=[run.ctx])
                else:
                    plan.run_mine(kind, ctxs=[ctx])
            return {j: plan.get_result(kind, j) for j in mine}

        if untagged:
            got = [None] * world
            dist.all_gather_object(got, run(JOB_HAPTAG), group=group)
            for r, part in enumerate(got):
                if r != rank:
                    for j, res in part.items():
                        plan.set_result(JOB_HAPTAG, j, res)
            plan.merge_raw()
        mine = run(JOB_WINDOWS)
        got = [None] * world if rank == writer else None
        dist.gather_object(mine, got, dst=writer, group=group)
        out = [None]
        if rank == writer:
            for r, part in enumerate(got):
                if r != rank:
                    for j, res in part.items():
                        plan.set_result(JOB_WINDOWS, j, res)
            plan.finish()
            out = [_result(plan, mode)]
        dist.broadcast_object_list(out, src=writer, group=group)
        return out[0]
    finally:
        if getattr(run, "ctx", None) is not None:
            run.ctx.close()
        plan.close()

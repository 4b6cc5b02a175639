"""Host BAM ingest: pf_bam_* of libpomfret_amd.so.

`BamFile(path).fetch_windows(chrom, starts, ends)` returns the records the
reference's load_reads_given_interval fetches for each window
(blockjoin.c:1053-1076: region ``chrom:max(s-readback,0)-(e+readback)``,
htslib region/overlap semantics) as an `AlnBatch` ready for
`Context.upload_aln`, plus each record's qname (for the first-wins tag
table of blockjoin.c:4408-4423).  Host code; no GPU involved.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ._lib import PomfretError, _check, lib
from .abi import AlnBatch, KnownVars, PfAlnBatch, PfKnownVars, ReadAlnBatch

READBACK = 50_000  # blockjoin.c READBACK, the region margin of 1053-1054


class PfBamRecords(C.Structure):
    _fields_ = [("aln", PfAlnBatch), ("qname_off", C.c_void_p), ("qname", C.c_void_p),
                ("hp_tag", C.c_void_p), ("n_truncated", C.c_uint64)]


class PfReadAlnBatch(C.Structure):
    _fields_ = [("n_reads", C.c_uint32)] + [(n, C.c_void_p) for n in (
        "start", "end", "cigar_off", "cigar", "seq_off", "seq_len", "seq", "md_off", "md")]


class PfBamReads(C.Structure):
    _fields_ = [("reads", PfReadAlnBatch), ("qname_off", C.c_void_p), ("qname", C.c_void_p),
                ("n_truncated", C.c_uint64)]


class PfKnownTable(C.Structure):
    _fields_ = [("vars", PfKnownVars)]


class PfQnameTags(C.Structure):
    _fields_ = [("n", C.c_uint32), ("off", C.c_void_p), ("names", C.c_void_p), ("hp", C.c_void_p)]


class PfRescueMap(C.Structure):
    _fields_ = [("n", C.c_uint32), ("pos", C.c_void_p), ("hap_of_ref", C.c_void_p)]


_bound = False


class PfBamDevFetch(C.Structure):
    _fields_ = [("n_windows", C.c_uint32), ("n_recs", C.c_uint64), ("win_rec_off", C.c_void_p),
                ("win_n_fetched", C.c_void_p), ("qname_off", C.c_void_p), ("qname", C.c_void_p),
                ("hp_tag", C.c_void_p), ("n_truncated", C.c_uint64), ("comp_bytes", C.c_uint64),
                ("inflated_bytes", C.c_uint64), ("n_blocks", C.c_uint64), ("n_chain_recs", C.c_uint64),
                ("ms_read", C.c_double), ("ms_inflate", C.c_double), ("ms_chain", C.c_double),
                ("ms_decode", C.c_double), ("ms_select", C.c_double), ("ms_build", C.c_double),
                ("ms_total", C.c_double), ("attempts", C.c_uint32), ("read_hp", C.c_void_p),
                ("from_arena", C.c_uint32)]


def _bind():
    global _bound
    if _bound:
        return lib()
    L = lib()
    L.pf_bam_open.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_void_p)]
    L.pf_bam_close.argtypes = [C.c_void_p]
    L.pf_bam_n_targets.argtypes = [C.c_void_p]
    L.pf_bam_n_targets.restype = C.c_int32
    L.pf_bam_target_name.argtypes = [C.c_void_p, C.c_int32]
    L.pf_bam_target_name.restype = C.c_char_p
    L.pf_bam_target_len.argtypes = [C.c_void_p, C.c_int32]
    L.pf_bam_target_len.restype = C.c_uint32
    L.pf_bam_tid.argtypes = [C.c_void_p, C.c_char_p]
    L.pf_bam_tid.restype = C.c_int32
    L.pf_bam_index_stats.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.pf_bam_fetch_windows.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                       C.c_uint32, C.c_int, C.POINTER(C.POINTER(PfBamRecords))]
    L.pf_bam_records_free.argtypes = [C.POINTER(PfBamRecords)]
    L.pf_bam_fetch_contig_reads.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.POINTER(PfBamReads))]
    L.pf_bam_reads_free.argtypes = [C.POINTER(PfBamReads)]
    L.pf_vcf_known_vars.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.POINTER(PfKnownTable))]
    L.pf_known_table_free.argtypes = [C.POINTER(PfKnownTable)]
    L.pf_rescue_dropped.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                    C.POINTER(PfKnownVars), C.POINTER(PfQnameTags), C.POINTER(PfQnameTags),
                                    C.POINTER(C.POINTER(PfRescueMap))]
    L.pf_rescue_dropped_mt.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                       C.POINTER(PfKnownVars), C.POINTER(PfQnameTags), C.POINTER(PfQnameTags),
                                       C.c_int, C.POINTER(C.POINTER(PfRescueMap))]
    L.pf_rescue_map_free.argtypes = [C.POINTER(PfRescueMap)]
    L.pf_bam_estimate_coverage.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
    L.pf_bam_set_threads.argtypes = [C.c_void_p, C.c_int]
    L.pf_bam_set_threads.restype = None
    L.pf_bam_estimate_coverage_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_uint64]
    L.pf_bam_n_no_coor.argtypes = [C.c_void_p]
    L.pf_bam_n_no_coor.restype = C.c_int64
    L.pf_bam_query_chunks.argtypes = [C.c_void_p, C.c_int32, C.c_int64, C.c_int64, C.c_void_p, C.c_uint64]
    L.pf_bam_query_chunks.restype = C.c_int64
    L.pf_batch_upload_bam.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_char_p, C.c_uint32,
                                      C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_void_p),
                                      C.POINTER(C.POINTER(PfBamDevFetch))]
    L.pf_bam_dev_fetch_free.argtypes = [C.POINTER(PfBamDevFetch)]
    L.pf_haptag_bam.argtypes = [C.c_void_p, C.POINTER(PfKnownVars), C.c_void_p, C.c_char_p,
                                C.POINTER(C.POINTER(PfBamDevFetch))]
    _bound = True
    return L


def _arr(ptr, n, dt) -> np.ndarray:
    n = int(n)
    if n == 0 or not ptr:
        return np.zeros(0, dt)
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dt))), (n,)).copy()


class BamFile:
    """An opened BAM + BAI (pf_bam_open).  bam=None opens the index alone."""

    def __init__(self, bam: Optional[str], bai: Optional[str] = None, threads: int = 1):
        """threads: BGZF inflate threads of the sequential passes
        (estimate_coverage, fetch_contig_reads; pf_bam_set_threads) -- the
        reference's -t N for bgzf_mt (blockjoin.c:576-578)."""
        L = _bind()
        h = C.c_void_p()
        rc = L.pf_bam_open(bam.encode() if bam else None, bai.encode() if bai else None, C.byref(h))
        if rc == -1:
            raise FileNotFoundError(bam or bai)
        _check(rc, "pf_bam_open")
        self.handle = h
        self.path = bam
        if threads > 1:
            L.pf_bam_set_threads(h, int(threads))

    def close(self):
        if self.handle:
            lib().pf_bam_close(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def n_targets(self) -> int:
        return int(lib().pf_bam_n_targets(self.handle))

    @property
    def targets(self) -> List[str]:
        return [lib().pf_bam_target_name(self.handle, i).decode() for i in range(self.n_targets)]

    @property
    def lengths(self) -> List[int]:
        return [int(lib().pf_bam_target_len(self.handle, i)) for i in range(self.n_targets)]

    def tid(self, name: str) -> int:
        return int(lib().pf_bam_tid(self.handle, name.encode()))

    def index_stats(self, tid: int) -> Tuple[int, int]:
        """(mapped, unmapped) of the BAI's metadata pseudo-bin."""
        m, u = C.c_uint64(), C.c_uint64()
        _check(lib().pf_bam_index_stats(self.handle, int(tid), C.byref(m), C.byref(u)), "pf_bam_index_stats")
        return int(m.value), int(u.value)

    def fetch_windows(self, chrom: str, starts: Sequence[int], ends: Sequence[int],
                      readback: int = READBACK, threads: int = 1) -> Tuple[AlnBatch, List[str], dict]:
        """The records of every window [s, e] (gap coordinates as the
        methphase worker receives them) -> (AlnBatch, qnames, info)."""
        if self.path is None:
            raise PomfretError("index-only BamFile cannot fetch")
        L = _bind()
        ws = np.ascontiguousarray(starts, np.uint32)
        we = np.ascontiguousarray(ends, np.uint32)
        if ws.shape != we.shape:
            raise ValueError("starts and ends differ in length")
        out = C.POINTER(PfBamRecords)()
        _check(L.pf_bam_fetch_windows(self.handle, chrom.encode(), ws.size, ws.ctypes.data, we.ctypes.data,
                                      int(readback), int(threads), C.byref(out)), "pf_bam_fetch_windows")
        try:
            r = out.contents
            a = r.aln
            n, W = int(a.n_recs), int(a.n_windows)
            co = _arr(a.cigar_off, n + 1, np.uint64)
            so = _arr(a.seq_off, n + 1, np.uint64)
            mo = _arr(a.mm_off, n + 1, np.uint64)
            lo = _arr(a.ml_off, n + 1, np.uint64)
            qo = _arr(r.qname_off, n + 1, np.uint64)
            batch = AlnBatch(
                win_start=ws.copy(), win_end=we.copy(), win_rec_off=_arr(a.win_rec_off, W + 1, np.uint32),
                flag=_arr(a.flag, n, np.uint16), mapq=_arr(a.mapq, n, np.uint8), pos=_arr(a.pos, n, np.uint32),
                l_qseq=_arr(a.l_qseq, n, np.uint32), de=_arr(a.de, n, np.float32), hp=_arr(a.hp, n, np.uint8),
                cigar_off=co, cigar=_arr(a.cigar, co[-1], np.uint32),
                seq_off=so, seq=_arr(a.seq, so[-1], np.uint8),
                mm_off=mo, mm=_arr(a.mm, mo[-1], np.uint8),
                ml_off=lo, ml=_arr(a.ml, lo[-1], np.uint8))
            qb = _arr(r.qname, qo[-1], np.uint8).tobytes()
            qnames = [qb[qo[i]:qo[i + 1]].decode("ascii", "replace") for i in range(n)]
            info = {"hp_tag": _arr(r.hp_tag, n, np.int32), "n_truncated": int(r.n_truncated)}
        finally:
            L.pf_bam_records_free(out)
        return batch, qnames, info

    def query_chunks(self, chrom: str, beg: int, end: int) -> np.ndarray:
        """BAI chunks [u, v) of region [beg, end) (pf_bam_query_chunks), shape (n, 2)."""
        L = _bind()
        tid = self.tid(chrom)
        n = int(L.pf_bam_query_chunks(self.handle, tid, int(beg), int(end), None, 0))
        _check(min(n, 0), "pf_bam_query_chunks")
        out = np.zeros(2 * max(n, 1), np.uint64)
        L.pf_bam_query_chunks(self.handle, tid, int(beg), int(end), out.ctypes.data, n)
        return out[:2 * n].reshape(n, 2)

    def fetch_windows_device(self, ctx, cfg, chrom: str, starts: Sequence[int], ends: Sequence[int],
                             lcfg=None, readback: int = READBACK, max_win_recs: int = 0):
        """Device fetch (pf_batch_upload_bam): the windows' records inflated,
        selected and gathered on the GPU into a record-level batch.  Returns
        (DeviceBatch, qnames, info)."""
        from ._lib import DeviceBatch
        from .abi import LoadConfig
        if self.path is None:
            raise PomfretError("index-only BamFile cannot fetch")
        L = _bind()
        ws = np.ascontiguousarray(starts, np.uint32)
        we = np.ascontiguousarray(ends, np.uint32)
        c = cfg.to_c()
        lc = (lcfg or LoadConfig()).to_c()
        h = C.c_void_p()
        f = C.POINTER(PfBamDevFetch)()
        _check(L.pf_batch_upload_bam(ctx.handle, C.byref(c), C.byref(lc), self.handle, chrom.encode(), ws.size,
                                     ws.ctypes.data, we.ctypes.data, int(readback), int(max_win_recs), C.byref(h),
                                     C.byref(f)), "pf_batch_upload_bam")
        try:
            r = f.contents
            n, W = int(r.n_recs), int(r.n_windows)
            qo = _arr(r.qname_off, n + 1, np.uint64)
            qb = _arr(r.qname, qo[-1] if n else 0, np.uint8).tobytes()
            qnames = [qb[qo[i]:qo[i + 1]].decode("ascii", "replace") for i in range(n)]
            info = {k: getattr(r, k) for k, _ in PfBamDevFetch._fields_
                    if k not in ("win_rec_off", "win_n_fetched", "qname_off", "qname", "hp_tag", "read_hp")}
            info["win_rec_off"] = _arr(r.win_rec_off, W + 1, np.uint32)
            info["win_n_fetched"] = _arr(r.win_n_fetched, W, np.uint32)
            info["hp_tag"] = _arr(r.hp_tag, n, np.int32)
        finally:
            L.pf_bam_dev_fetch_free(f)
        return DeviceBatch._wrap(ctx, h, W), qnames, info

    def haptag_device(self, ctx, chrom: str, known) -> Tuple[np.ndarray, List[str], dict]:
        """The -u pre-pass of one contig through the device fetch
        (pf_haptag_bam): (tag per read, qnames, info), reads in BAM order."""
        if self.path is None:
            raise PomfretError("index-only BamFile cannot fetch")
        L = _bind()
        kc = known.to_c()
        f = C.POINTER(PfBamDevFetch)()
        _check(L.pf_haptag_bam(ctx.handle, C.byref(kc), self.handle, chrom.encode(), C.byref(f)), "pf_haptag_bam")
        try:
            r = f.contents
            n = int(r.n_recs)
            qo = _arr(r.qname_off, n + 1, np.uint64)
            qb = _arr(r.qname, qo[-1] if n else 0, np.uint8).tobytes()
            qnames = [qb[qo[i]:qo[i + 1]].decode("ascii", "replace") for i in range(n)]
            hp = _arr(r.read_hp, n, np.uint8)
            info = {k: getattr(r, k) for k, _ in PfBamDevFetch._fields_ if k.startswith("ms_") or k in
                    ("n_truncated", "comp_bytes", "inflated_bytes", "n_blocks", "n_chain_recs", "attempts")}
        finally:
            L.pf_bam_dev_fetch_free(f)
        return hp, qnames, info

    def estimate_coverage(self) -> List[int]:
        """estimate_read_coverage_dirtyfast (blockjoin.c:951-1040): per contig."""
        L = _bind()
        cov = np.zeros(max(self.n_targets, 1), np.int32)
        _check(L.pf_bam_estimate_coverage(self.handle, cov.ctypes.data, cov.size), "pf_bam_estimate_coverage")
        return cov[:self.n_targets].tolist()

    def estimate_coverage_device(self, ctx, piece_bytes: int = 0) -> List[int]:
        """The same estimate with the pass over the BAM on ctx's device
        (pf_bam_estimate_coverage_dev); piece_bytes bounds the compressed bytes
        of one fetch (0: 4 GiB)."""
        L = _bind()
        cov = np.zeros(max(self.n_targets, 1), np.int32)
        _check(L.pf_bam_estimate_coverage_dev(ctx.handle, self.handle, cov.ctypes.data, cov.size, piece_bytes),
               "pf_bam_estimate_coverage_dev")
        return cov[:self.n_targets].tolist()

    @property
    def n_unplaced(self) -> int:
        """The index's count of unplaced records (-1: not recorded)."""
        return int(_bind().pf_bam_n_no_coor(self.handle))

    def fetch_contig_reads(self, chrom: str) -> Tuple[ReadAlnBatch, List[str], dict]:
        """The -u pre-pass reads of one contig (pf_bam_fetch_contig_reads):
        primary mapped records with CIGAR, SEQ and MD, in BAM order."""
        if self.path is None:
            raise PomfretError("index-only BamFile cannot fetch")
        L = _bind()
        out = C.POINTER(PfBamReads)()
        _check(L.pf_bam_fetch_contig_reads(self.handle, chrom.encode(), C.byref(out)), "pf_bam_fetch_contig_reads")
        try:
            r = out.contents
            a = r.reads
            n = int(a.n_reads)
            co = _arr(a.cigar_off, n + 1, np.uint64)
            so = _arr(a.seq_off, n + 1, np.uint64)
            mo = _arr(a.md_off, n + 1, np.uint64)
            qo = _arr(r.qname_off, n + 1, np.uint64)
            reads = ReadAlnBatch(start=_arr(a.start, n, np.uint32), end=_arr(a.end, n, np.uint32),
                                 cigar_off=co, cigar=_arr(a.cigar, co[-1], np.uint32),
                                 seq_off=so, seq_len=_arr(a.seq_len, n, np.uint32), seq=_arr(a.seq, so[-1], np.uint8),
                                 md_off=mo, md=_arr(a.md, mo[-1], np.uint8))
            qb = _arr(r.qname, qo[-1], np.uint8).tobytes()
            qnames = [qb[qo[i]:qo[i + 1]].decode("ascii", "replace") for i in range(n)]
            info = {"n_truncated": int(r.n_truncated)}
        finally:
            L.pf_bam_reads_free(out)
        return reads, qnames, info


def _known_of(L, t) -> KnownVars:
    try:
        v = t.contents.vars
        n = int(v.n)
        off = _arr(v.char_off, n + 1, np.uint64)
        return KnownVars(pos=_arr(v.pos, n, np.uint32), len=_arr(v.len, n, np.uint32), op=_arr(v.op, n, np.uint8),
                         haptag=_arr(v.haptag, n, np.uint8), char_off=off, chars=_arr(v.chars, off[-1], np.uint8))
    finally:
        L.pf_known_table_free(t)


def vcf_known_vars(vcf_path: str, contig: str) -> KnownVars:
    """The -u known-variant table of one contig (pf_vcf_known_vars)."""
    L = _bind()
    out = C.POINTER(PfKnownTable)()
    rc = L.pf_vcf_known_vars(vcf_path.encode(), contig.encode(), C.byref(out))
    if rc == -1:
        raise FileNotFoundError(vcf_path)
    _check(rc, "pf_vcf_known_vars")
    return _known_of(L, out)


def vcf_known_vars_multi(vcf_path: str, names) -> List[KnownVars]:
    """The rescue's known tables for the phase-block file's contigs in one
    pass (pf_vcf_known_vars_multi: a CHROM not among `names` goes to the
    table the previous line went to, blockjoin.c:2150-2163)."""
    L = _bind()
    n = len(names)
    enc = [x.encode() for x in names]
    arr = (C.c_char_p * max(n, 1))(*enc)
    outs = (C.POINTER(PfKnownTable) * max(n, 1))()
    L.pf_vcf_known_vars_multi.argtypes = [C.c_char_p, C.c_uint32, C.c_void_p, C.c_void_p]
    rc = L.pf_vcf_known_vars_multi(vcf_path.encode(), n, C.cast(arr, C.c_void_p), C.cast(outs, C.c_void_p))
    if rc == -1:
        raise FileNotFoundError(vcf_path)
    _check(rc, "pf_vcf_known_vars_multi")
    return [_known_of(L, outs[i]) for i in range(n)]


def _qname_tags(table: Dict[str, int]):
    """(PfQnameTags, keepalive) of a qname -> hp dict (insertion order)."""
    names = [q.encode() for q in table]
    off = np.zeros(len(names) + 1, np.uint64)
    if names:
        off[1:] = np.cumsum([len(q) for q in names])
    buf = np.frombuffer(b"".join(names) or b"\0", np.uint8).copy()
    hp = np.asarray([int(v) & 0xFF for v in table.values()] or [0], np.uint8)
    t = PfQnameTags(len(names), off.ctypes.data, buf.ctypes.data, hp.ctypes.data)
    return t, (off, buf, hp)


def rescue_dropped(bam: BamFile, contig: str, dropped, known: KnownVars, methphased: Dict[str, int],
                   raw: Optional[Dict[str, int]] = None, threads: int = 1) -> Dict[int, int]:
    """pf_rescue_dropped(_mt): {0-based pos: hap_of_ref} of one contig's
    dropped intervals [(s, e), ...] for the VCF writer (Blocks.write_vcf
    rescue); threads > 1 spreads the intervals over host threads."""
    L = _bind()
    ds = np.ascontiguousarray([a for a, _ in dropped] or [0], np.uint32)
    de = np.ascontiguousarray([b for _, b in dropped] or [0], np.uint32)
    tm, km = _qname_tags(methphased)
    tr, kr = _qname_tags(raw) if raw is not None else (None, None)
    kc = known.to_c()
    out = C.POINTER(PfRescueMap)()
    _check(L.pf_rescue_dropped_mt(bam.handle, contig.encode(), len(dropped), ds.ctypes.data, de.ctypes.data,
                                  C.byref(kc), C.byref(tm), C.byref(tr) if tr is not None else None, int(threads),
                                  C.byref(out)), "pf_rescue_dropped_mt")
    try:
        m = out.contents
        n = int(m.n)
        pos = _arr(m.pos, n, np.uint32)
        hap = _arr(m.hap_of_ref, n, np.uint8)
    finally:
        L.pf_rescue_map_free(out)
    del km, kr
    return {int(p): int(h) for p, h in zip(pos, hap)}


RETAG_METHPHASE, RETAG_VARHAPTAG = 0, 1


def retag_bam(bam_in: str, bam_out: Optional[str], bai_out: Optional[str], tsv_out: Optional[str], mode: int,
              gaps=None, blocks=None, methphased=None, raw=None, level: int = -1, threads: int = 1) -> int:
    """pf_retag_bam_threads: --write-bam (mode RETAG_METHPHASE,
    output_modify_bam) or varhaptag (RETAG_VARHAPTAG) output of bam_in.  gaps /
    blocks: _lib.Gaps / _lib.Blocks; methphased / raw: pipeline.Tags (or
    None); threads: BGZF compression threads (-T).  Returns the number of
    records written."""
    from ._lib import _PfBlocks, _PfGaps
    L = _bind()
    if not getattr(L, "_retag_typed", False):
        L.pf_retag_bam_threads.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_int,
                                           C.POINTER(_PfGaps), C.POINTER(_PfBlocks), C.c_void_p, C.c_void_p, C.c_int,
                                           C.c_int, C.POINTER(C.c_uint64)]
        L._retag_typed = True
    n = C.c_uint64()
    enc = lambda s: s.encode() if s else None  # noqa: E731
    _check(L.pf_retag_bam_threads(enc(bam_in), enc(bam_out), enc(bai_out), enc(tsv_out), int(mode),
                                  gaps._p if gaps is not None else None, blocks._p if blocks is not None else None,
                                  methphased.h if methphased is not None else None, raw.h if raw is not None else None,
                                  int(level), int(threads), C.byref(n)), "pf_retag_bam_threads")
    return int(n.value)

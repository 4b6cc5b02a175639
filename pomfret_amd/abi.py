"""ctypes mirror of include/pomfret_amd.h plus numpy-side batch containers.

This module only describes the C ABI; it never computes anything.  The
product entry points live in pomfret_amd/_lib.py (libpomfret_amd.so); the CPU
oracle (tests / bench baseline only) reuses these struct definitions.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

PF_OK = 0
PF_ERR_ARG = -1
PF_ERR_HIP = -2
PF_ERR_NOMEM = -3
PF_ERR_UNSUPPORTED = -4
PF_ERR_LIMIT = -5
PF_ERR_INTERNAL = -6

HAPTAG_UNPHASED = 254  # reference blockjoin.c:26


class PfCfg(C.Structure):
    """pf_cfg_t  (mirrors mmr_config_t, reference blockjoin.h:7-16)."""
    _fields_ = [
        ("k", C.c_int32),
        ("k_span", C.c_int32),
        ("cov_for_selection", C.c_int32),
        ("cov_for_runtime", C.c_int32),
        ("n_cand", C.c_int32),
        ("hard_cov", C.c_int32),
        ("flags", C.c_int32),
        ("reserved", C.c_int32),
    ]


class PfWindowBatch(C.Structure):
    _fields_ = [
        ("n_windows", C.c_uint32),
        ("n_reads", C.c_uint32),
        ("n_calls", C.c_uint64),
        ("win_start", C.c_void_p),
        ("win_end", C.c_void_p),
        ("win_read_off", C.c_void_p),
        ("win_cov_sel", C.c_void_p),
        ("win_cov_rt", C.c_void_p),
        ("win_n_cand", C.c_void_p),
        ("read_start", C.c_void_p),
        ("read_end", C.c_void_p),
        ("read_hp", C.c_void_p),
        ("read_call_off", C.c_void_p),
        ("call_pos", C.c_void_p),
        ("call_cat", C.c_void_p),
    ]


class PfWindowOut(C.Structure):
    _fields_ = [
        ("decision", C.c_void_p),
        ("read_hp", C.c_void_p),
        ("dir_table", C.c_void_p),
        ("dir_join", C.c_void_p),
        ("dir_which_way", C.c_void_p),
        ("dir_fisher_p", C.c_void_p),
        ("dir_score", C.c_void_p),
        ("win_n_sites", C.c_void_p),
        ("win_n_reads", C.c_void_p),
    ]


class PfKnownVars(C.Structure):
    _fields_ = [
        ("n", C.c_uint32),
        ("pos", C.c_void_p),
        ("len", C.c_void_p),
        ("op", C.c_void_p),
        ("haptag", C.c_void_p),
        ("char_off", C.c_void_p),
        ("chars", C.c_void_p),
    ]


class PfReadAlnBatch(C.Structure):
    _fields_ = [
        ("n_reads", C.c_uint32),
        ("start", C.c_void_p),
        ("end", C.c_void_p),
        ("cigar_off", C.c_void_p),
        ("cigar", C.c_void_p),
        ("seq_off", C.c_void_p),
        ("seq_len", C.c_void_p),
        ("seq", C.c_void_p),
        ("md_off", C.c_void_p),
        ("md", C.c_void_p),
    ]


def _ptr(a: Optional[np.ndarray]) -> Optional[int]:
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays must be C-contiguous"
    return a.ctypes.data


@dataclass
class Config:
    """Hot-path parameters.  Defaults = `pomfret methphase -c 60` (cli.c:270-275,
    blockjoin.c:4656-4659): cov_for_selection 6, cov_for_runtime 12, n_cand 15."""
    k: int = 3
    k_span: int = 5000
    cov_for_selection: int = 6
    cov_for_runtime: int = 12
    n_cand: int = 15
    hard_cov: int = 15

    @staticmethod
    def from_coverage(cov: int, report: bool = False, given: bool = True) -> "Config":
        """Parameter derivation of the reference.
        methphase -c C   : C/10, 2*(C/10), C/4          (cli.c:270-275, blockjoin.c:4657)
        methphase (auto) : est/10+1, 2*(...), est/4+1   (blockjoin.c:4373-4375)
        report           : c/10+1, 2*(...), c/4+1       (blockjoin.c:5045-5051)
        followed by the clamps of blockjoin.c:4381-4390."""
        if report or not given:
            sel, nc = cov // 10 + 1, cov // 4 + 1
        else:
            sel, nc = cov // 10, cov // 4
        rt = 2 * sel
        if sel <= 0:
            sel = 1
        if nc <= 1:
            nc = 2
        return Config(cov_for_selection=sel, cov_for_runtime=rt, n_cand=nc)

    def to_c(self) -> PfCfg:
        return PfCfg(self.k, self.k_span, self.cov_for_selection, self.cov_for_runtime,
                     self.n_cand, self.hard_cov, 0, 0)


@dataclass
class WindowBatch:
    """Host SoA of a batch of windows (see pf_window_batch_t)."""
    win_start: np.ndarray      # u32 [W]
    win_end: np.ndarray        # u32 [W]
    win_read_off: np.ndarray   # u32 [W+1]
    read_start: np.ndarray     # u32 [R]
    read_end: np.ndarray       # u32 [R]
    read_hp: np.ndarray        # u8  [R]
    read_call_off: np.ndarray  # u64 [R+1]
    call_pos: np.ndarray       # u32 [N]
    call_cat: np.ndarray       # u8  [N]
    win_cov_sel: Optional[np.ndarray] = None  # i32 [W]
    win_cov_rt: Optional[np.ndarray] = None
    win_n_cand: Optional[np.ndarray] = None
    meta: dict = field(default_factory=dict)

    def __post_init__(self):
        self.win_start = np.ascontiguousarray(self.win_start, dtype=np.uint32)
        self.win_end = np.ascontiguousarray(self.win_end, dtype=np.uint32)
        self.win_read_off = np.ascontiguousarray(self.win_read_off, dtype=np.uint32)
        self.read_start = np.ascontiguousarray(self.read_start, dtype=np.uint32)
        self.read_end = np.ascontiguousarray(self.read_end, dtype=np.uint32)
        self.read_hp = np.ascontiguousarray(self.read_hp, dtype=np.uint8)
        self.read_call_off = np.ascontiguousarray(self.read_call_off, dtype=np.uint64)
        self.call_pos = np.ascontiguousarray(self.call_pos, dtype=np.uint32)
        self.call_cat = np.ascontiguousarray(self.call_cat, dtype=np.uint8)
        for name in ("win_cov_sel", "win_cov_rt", "win_n_cand"):
            v = getattr(self, name)
            if v is not None:
                setattr(self, name, np.ascontiguousarray(v, dtype=np.int32))

    @property
    def n_windows(self) -> int:
        return int(self.win_start.shape[0])

    @property
    def n_reads(self) -> int:
        return int(self.read_start.shape[0])

    @property
    def n_calls(self) -> int:
        return int(self.call_pos.shape[0])

    def to_c(self) -> PfWindowBatch:
        b = PfWindowBatch()
        b.n_windows = self.n_windows
        b.n_reads = self.n_reads
        b.n_calls = self.n_calls
        b.win_start = _ptr(self.win_start)
        b.win_end = _ptr(self.win_end)
        b.win_read_off = _ptr(self.win_read_off)
        b.win_cov_sel = _ptr(self.win_cov_sel)
        b.win_cov_rt = _ptr(self.win_cov_rt)
        b.win_n_cand = _ptr(self.win_n_cand)
        b.read_start = _ptr(self.read_start)
        b.read_end = _ptr(self.read_end)
        b.read_hp = _ptr(self.read_hp)
        b.read_call_off = _ptr(self.read_call_off)
        b.call_pos = _ptr(self.call_pos)
        b.call_cat = _ptr(self.call_cat)
        return b

    def select(self, windows) -> "WindowBatch":
        """Sub-batch with the given window indices (reads/calls re-packed)."""
        windows = np.asarray(windows, dtype=np.int64)
        ro = self.win_read_off.astype(np.int64)
        co = self.read_call_off.astype(np.int64)
        reads = [np.arange(ro[w], ro[w + 1]) for w in windows]
        reads = np.concatenate(reads) if reads else np.zeros(0, np.int64)
        rcount = np.array([ro[w + 1] - ro[w] for w in windows], dtype=np.int64)
        ccount = co[reads + 1] - co[reads]
        calls = [np.arange(co[r], co[r + 1]) for r in reads]
        calls = np.concatenate(calls) if len(calls) else np.zeros(0, np.int64)
        sub = lambda a: None if a is None else a[windows]
        return WindowBatch(
            win_start=self.win_start[windows], win_end=self.win_end[windows],
            win_read_off=np.concatenate([[0], np.cumsum(rcount)]),
            read_start=self.read_start[reads], read_end=self.read_end[reads],
            read_hp=self.read_hp[reads],
            read_call_off=np.concatenate([[0], np.cumsum(ccount)]),
            call_pos=self.call_pos[calls], call_cat=self.call_cat[calls],
            win_cov_sel=sub(self.win_cov_sel), win_cov_rt=sub(self.win_cov_rt),
            win_n_cand=sub(self.win_n_cand), meta=dict(self.meta))


@dataclass
class WindowResult:
    decision: np.ndarray      # i8  [W]
    read_hp: np.ndarray       # u8  [R]
    dir_table: np.ndarray     # i32 [W,2,4]
    dir_join: np.ndarray      # i32 [W,2]
    dir_which_way: np.ndarray # i32 [W,2]
    dir_fisher_p: np.ndarray  # f64 [W,2]
    dir_score: np.ndarray     # f32 [W,2]
    win_n_sites: np.ndarray   # u32 [W]
    win_n_reads: np.ndarray   # u32 [W]

    @staticmethod
    def alloc(n_windows: int, n_reads: int) -> "WindowResult":
        W, R = n_windows, n_reads
        return WindowResult(
            decision=np.full(W, -2, np.int8), read_hp=np.full(R, 255, np.uint8),
            dir_table=np.full((W, 2, 4), -1, np.int32), dir_join=np.full((W, 2), -5, np.int32),
            dir_which_way=np.full((W, 2), -5, np.int32), dir_fisher_p=np.full((W, 2), -1.0),
            dir_score=np.full((W, 2), -1.0, np.float32), win_n_sites=np.zeros(W, np.uint32),
            win_n_reads=np.zeros(W, np.uint32))

    def to_c(self) -> PfWindowOut:
        o = PfWindowOut()
        o.decision = _ptr(self.decision)
        o.read_hp = _ptr(self.read_hp)
        o.dir_table = _ptr(self.dir_table)
        o.dir_join = _ptr(self.dir_join)
        o.dir_which_way = _ptr(self.dir_which_way)
        o.dir_fisher_p = _ptr(self.dir_fisher_p)
        o.dir_score = _ptr(self.dir_score)
        o.win_n_sites = _ptr(self.win_n_sites)
        o.win_n_reads = _ptr(self.win_n_reads)
        return o


@dataclass
class KnownVars:
    pos: np.ndarray       # u32
    len: np.ndarray       # u32
    op: np.ndarray        # u8
    haptag: np.ndarray    # u8
    char_off: np.ndarray  # u64 [n+1]
    chars: np.ndarray     # u8

    def __post_init__(self):
        self.pos = np.ascontiguousarray(self.pos, np.uint32)
        self.len = np.ascontiguousarray(self.len, np.uint32)
        self.op = np.ascontiguousarray(self.op, np.uint8)
        self.haptag = np.ascontiguousarray(self.haptag, np.uint8)
        self.char_off = np.ascontiguousarray(self.char_off, np.uint64)
        self.chars = np.ascontiguousarray(self.chars if len(self.chars) else np.zeros(1, np.uint8), np.uint8)

    def to_c(self) -> PfKnownVars:
        k = PfKnownVars()
        k.n = int(self.pos.shape[0])
        k.pos, k.len, k.op, k.haptag = _ptr(self.pos), _ptr(self.len), _ptr(self.op), _ptr(self.haptag)
        k.char_off, k.chars = _ptr(self.char_off), _ptr(self.chars)
        return k


@dataclass
class ReadAlnBatch:
    start: np.ndarray      # u32
    end: np.ndarray        # u32
    cigar_off: np.ndarray  # u64
    cigar: np.ndarray      # u32
    seq_off: np.ndarray    # u64
    seq_len: np.ndarray    # u32
    seq: np.ndarray        # u8 packed nibbles
    md_off: np.ndarray     # u64
    md: np.ndarray         # u8 (ASCII)

    def __post_init__(self):
        self.start = np.ascontiguousarray(self.start, np.uint32)
        self.end = np.ascontiguousarray(self.end, np.uint32)
        self.cigar_off = np.ascontiguousarray(self.cigar_off, np.uint64)
        self.cigar = np.ascontiguousarray(self.cigar if len(self.cigar) else np.zeros(1, np.uint32), np.uint32)
        self.seq_off = np.ascontiguousarray(self.seq_off, np.uint64)
        self.seq_len = np.ascontiguousarray(self.seq_len, np.uint32)
        self.seq = np.ascontiguousarray(self.seq if len(self.seq) else np.zeros(1, np.uint8), np.uint8)
        self.md_off = np.ascontiguousarray(self.md_off, np.uint64)
        self.md = np.ascontiguousarray(self.md if len(self.md) else np.zeros(1, np.uint8), np.uint8)

    @property
    def n_reads(self) -> int:
        return int(self.start.shape[0])

    def to_c(self) -> PfReadAlnBatch:
        r = PfReadAlnBatch()
        r.n_reads = self.n_reads
        r.start, r.end = _ptr(self.start), _ptr(self.end)
        r.cigar_off, r.cigar = _ptr(self.cigar_off), _ptr(self.cigar)
        r.seq_off, r.seq_len, r.seq = _ptr(self.seq_off), _ptr(self.seq_len), _ptr(self.seq)
        r.md_off, r.md = _ptr(self.md_off), _ptr(self.md)
        return r


class PfLoadCfg(C.Structure):
    """pf_load_cfg_t (mmr_config_t's loader fields, reference blockjoin.h:7-16)."""
    _fields_ = [("min_mapq", C.c_int32), ("min_len", C.c_int32),
                ("qual_lo", C.c_int32), ("qual_hi", C.c_int32)]


@dataclass
class LoadConfig:
    """Loader parameters; defaults are the CLI's (cli.c:56-70): -q 10, -L 15000,
    ML bands lo 100 / hi 156."""
    min_mapq: int = 10
    min_len: int = 15000
    qual_lo: int = 100
    qual_hi: int = 156

    def to_c(self) -> PfLoadCfg:
        return PfLoadCfg(self.min_mapq, self.min_len, self.qual_lo, self.qual_hi)


class PfAlnBatch(C.Structure):
    _fields_ = [("n_windows", C.c_uint32), ("n_recs", C.c_uint32)] + [
        (n, C.c_void_p) for n in (
            "win_start", "win_end", "win_rec_off", "win_cov_sel", "win_cov_rt", "win_n_cand",
            "flag", "mapq", "pos", "l_qseq", "de", "hp", "cigar_off", "cigar", "seq_off", "seq",
            "mm_off", "mm", "ml_off", "ml")]


_ALN_FIELDS = {
    "win_start": np.uint32, "win_end": np.uint32, "win_rec_off": np.uint32,
    "flag": np.uint16, "mapq": np.uint8, "pos": np.uint32, "l_qseq": np.uint32, "de": np.float32,
    "hp": np.uint8, "cigar_off": np.uint64, "cigar": np.uint32, "seq_off": np.uint64, "seq": np.uint8,
    "mm_off": np.uint64, "mm": np.uint8, "ml_off": np.uint64, "ml": np.uint8,
}


@dataclass
class AlnBatch:
    """Record-level host SoA of a batch of windows (pf_aln_batch_t): the BAM
    records each window's region query returned, in BAM order."""
    win_start: np.ndarray
    win_end: np.ndarray
    win_rec_off: np.ndarray
    flag: np.ndarray
    mapq: np.ndarray
    pos: np.ndarray
    l_qseq: np.ndarray
    de: np.ndarray
    hp: np.ndarray
    cigar_off: np.ndarray
    cigar: np.ndarray
    seq_off: np.ndarray
    seq: np.ndarray
    mm_off: np.ndarray
    mm: np.ndarray
    ml_off: np.ndarray
    ml: np.ndarray
    win_cov_sel: Optional[np.ndarray] = None
    win_cov_rt: Optional[np.ndarray] = None
    win_n_cand: Optional[np.ndarray] = None
    meta: dict = field(default_factory=dict)

    def __post_init__(self):
        for name, dt in _ALN_FIELDS.items():
            a = np.ascontiguousarray(getattr(self, name), dtype=dt)
            if name in ("cigar", "seq", "mm", "ml") and a.size == 0:
                a = np.zeros(1, dt)      # keep a valid pointer for empty arenas
            setattr(self, name, a)
        for name in ("win_cov_sel", "win_cov_rt", "win_n_cand"):
            v = getattr(self, name)
            if v is not None:
                setattr(self, name, np.ascontiguousarray(v, dtype=np.int32))

    @property
    def n_windows(self) -> int:
        return int(self.win_start.shape[0])

    @property
    def n_recs(self) -> int:
        return int(self.pos.shape[0])

    def to_c(self) -> PfAlnBatch:
        b = PfAlnBatch()
        b.n_windows = self.n_windows
        b.n_recs = self.n_recs
        for name in _ALN_FIELDS:
            setattr(b, name, _ptr(getattr(self, name)))
        for name in ("win_cov_sel", "win_cov_rt", "win_n_cand"):
            setattr(b, name, _ptr(getattr(self, name)))
        return b

    def nbytes(self) -> int:
        return int(sum(getattr(self, n).nbytes for n in _ALN_FIELDS))

    def select(self, windows) -> "AlnBatch":
        """Sub-batch with the given window indices (records re-packed)."""
        windows = np.asarray(windows, dtype=np.int64)
        wo = self.win_rec_off.astype(np.int64)
        recs = [np.arange(wo[w], wo[w + 1]) for w in windows]
        recs = np.concatenate(recs) if recs else np.zeros(0, np.int64)
        cnt = np.array([wo[w + 1] - wo[w] for w in windows], dtype=np.int64)

        def gather(off, data):
            off = np.asarray(off, np.int64)
            lo, hi = off[recs], off[recs + 1]
            sizes = hi - lo
            noff = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
            parts = [data[a:b] for a, b in zip(lo.tolist(), hi.tolist())]
            return noff, (np.concatenate(parts) if parts else data[:0])

        co, cg = gather(self.cigar_off, self.cigar)
        lq = self.l_qseq.astype(np.int64)
        so = np.asarray(self.seq_off, np.int64)
        sparts = [self.seq[so[r]:so[r] + (lq[r] + 1) // 2] for r in recs.tolist()]
        sq = np.concatenate(sparts) if sparts else self.seq[:0]
        soff = np.concatenate([[0], np.cumsum([(lq[r] + 1) // 2 for r in recs.tolist()])]).astype(np.uint64)
        mo, mm = gather(self.mm_off, self.mm)
        lo_, ml = gather(self.ml_off, self.ml)
        opt = {n: (None if getattr(self, n) is None else getattr(self, n)[windows])
               for n in ("win_cov_sel", "win_cov_rt", "win_n_cand")}
        return AlnBatch(win_start=self.win_start[windows], win_end=self.win_end[windows],
                        win_rec_off=np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32),
                        flag=self.flag[recs], mapq=self.mapq[recs], pos=self.pos[recs], l_qseq=self.l_qseq[recs],
                        de=self.de[recs], hp=self.hp[recs], cigar_off=co, cigar=cg, seq_off=soff, seq=sq,
                        mm_off=mo, mm=mm, ml_off=lo_, ml=ml, **opt)

"""Record-level (BAM field) inputs for the loader tests: hand-made records
with hand-worked expected calls, and seeded synthetic batches (synth_aln.py).

Every expected call list below is worked out from the reference's loops
(blockjoin.c line numbers in each comment), not from either implementation.
"""
import re

import numpy as np

from pomfret_amd.abi import AlnBatch, LoadConfig
from pomfret_amd.synth_aln import AlnSpec, make_aln_batch

_NT16 = {c: i for i, c in enumerate("=ACMGRSVTWYHKDBN")}
_OPS = {c: i for i, c in enumerate("MIDNSHP=X")}


def pack_seq(s: str) -> np.ndarray:
    codes = [_NT16[c] for c in s] + ([0] if len(s) % 2 else [])
    return np.array([(codes[i] << 4) | codes[i + 1] for i in range(0, len(codes), 2)], np.uint8)


def cigar_of(s: str) -> np.ndarray:
    return np.array([(int(n) << 4) | _OPS[op] for n, op in re.findall(r"(\d+)([MIDNSHP=X])", s)], np.uint32)


def records_batch(windows, **win_kw) -> AlnBatch:
    """windows: list of (s, e, [record dict]); record keys: seq, cigar, mm, ml,
    pos, flag, mapq, de, hp (defaults: flag 0, mapq 60, de 0.05, hp 0)."""
    recs = [r for _, _, rs in windows for r in rs]
    seqs = [pack_seq(r["seq"]) for r in recs]
    cigs = [cigar_of(r["cigar"]) for r in recs]
    mms = [np.frombuffer(r.get("mm", "").encode(), np.uint8) for r in recs]
    mls = [np.asarray(r.get("ml", []), np.uint8) for r in recs]

    def off(xs):
        return np.concatenate([[0], np.cumsum([x.shape[0] for x in xs])]).astype(np.uint64)

    def cat(xs, dt):
        return np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)

    return AlnBatch(
        win_start=[w[0] for w in windows], win_end=[w[1] for w in windows],
        win_rec_off=np.concatenate([[0], np.cumsum([len(w[2]) for w in windows])]),
        flag=[r.get("flag", 0) for r in recs], mapq=[r.get("mapq", 60) for r in recs],
        pos=[r["pos"] for r in recs], l_qseq=[len(r["seq"]) for r in recs],
        de=[r.get("de", 0.05) for r in recs], hp=[r.get("hp", 0) for r in recs],
        cigar_off=off(cigs), cigar=cat(cigs, np.uint32), seq_off=off(seqs), seq=cat(seqs, np.uint8),
        mm_off=off(mms), mm=cat(mms, np.uint8), ml_off=off(mls), ml=cat(mls, np.uint8), **win_kw)


# (name, record, expected calls [(ref pos, category)] or None when dropped)
HANDMADE = [
    # forward read, explicit calls at CpG C's; ref = pos + read offset (605-792)
    ("fwd", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0,0;", ml=[200, 10], pos=100),
     [(101, 0), (105, 1)]),
    # reverse read: the original read's C's are the stored G's counted from the
    # end; cgoffset -1 moves each call from the G to the CpG's C (618, 703)
    ("rev", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0,0;", ml=[50, 220], pos=200, flag=16),
     [(201, 0), (205, 1)]),
    # leading soft clip: a call on the first aligned base is pushed at qs+cgoffset
    # (640-648); a call on the first inserted base is consumed by the M op before
    # it (while i_read+length >= next_trigger, 663) and lands after the M block;
    # the deletion shifts the later call (offset += 2, 763)
    ("clip_ins_del", dict(seq="TTCGAACGTTACGA", cigar="2S4M1I2M2D5M", mm="C+m?,0,0,0;", ml=[255, 0, 130],
                          pos=1000),
     [(1000, 0), (1004, 1), (1010, 2)]),
    # implicit mode: a 5mC call outside CpG (the C at 7) sets has_implicit
    # (852-858); every other CpG C inside M ops becomes an unmethylated call
    # (666-700, 727-761)
    ("implicit", dict(seq="ACGACGTCAGCG", cigar="12M", mm="C+m?,1,0;", ml=[220, 30], pos=500),
     [(501, 1), (504, 0), (510, 1)]),
    # every call inside the leading soft clip: the exhausted trigger stays
    # "next" and the first M op pushes it (629-652 then 663-710)
    ("stale", dict(seq="ACGAAAAAA", cigar="3S6M", mm="C+m?,0;", ml=[250], pos=300), [(298, 0)]),
    # ... and with implicit mode the canonical scan restarts behind the stale call
    ("stale_implicit", dict(seq="ACGACAACGAA", cigar="5S6M", mm="C+m?,0,0;", ml=[200, 200], pos=400),
     [(396, 0), (402, 1)]),
    # 5hmC entry first: the 5mC ML values start after it (htslib ML order)
    ("h_then_m", dict(seq="ACGTTCGA", cigar="8M", mm="C+h?,0,0;C+m?,1;", ml=[5, 6, 180], pos=100),
     [(105, 0)]),
    # ChEBI-coded entry first, then 5mC
    ("chebi_then_m", dict(seq="ACGTTCGA", cigar="8M", mm="C+76792?,0;C+m?,0,0;", ml=[9, 99, 100], pos=100),
     [(101, 1), (105, 2)]),
    # combined codes: ML interleaved per position (h, m)
    ("combined_hm", dict(seq="ACGTTCGA", cigar="8M", mm="C+hm?,0,0;", ml=[1, 2, 3, 4], pos=100),
     [(101, 1), (105, 1)]),
    # several C m entries (duplex-style tags; round 5): htslib matches each
    # entry's canonical base against the read's base, whatever the strand, so
    # C-m counts the same C's as C+m; at one C the calls come in MM order and
    # get_mod_poss_on_ref keeps the last one's quality (846-880, 704-706)
    ("duplex_c_minus", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0;C-m?,0,0;", ml=[200, 10, 30], pos=100),
     [(101, 1), (105, 1)]),
    # G-m (the usual duplex encoding: the opposite strand's C) is not a C
    # entry: only its ML values are skipped
    ("duplex_g_minus", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0,0;G-m?,0,1;", ml=[200, 10, 5, 6], pos=100),
     [(101, 0), (105, 1)]),
    # a second C+m entry: its calls merge into the first's by position
    ("repeated_c_plus", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,1;C+m?,0;", ml=[180, 20], pos=100),
     [(101, 1), (105, 0)]),
    # reverse read: both entries count the stored G's from the end
    ("duplex_rev", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0;C-m?,1;", ml=[50, 220], pos=200, flag=16),
     [(201, 0), (205, 1)]),
    ("duplex_same_c_rev", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0,0;C-m?,0;", ml=[50, 220, 130], pos=200,
                               flag=16),
     [(201, 0), (205, 2)]),
    # no ML tag: quality 255 (HTS_MOD_UNKNOWN as uint8_t) -> methylated
    ("no_ml", dict(seq="ACGTTCGA", cigar="8M", mm="C+m.,0,0;", pos=100), [(101, 0), (105, 0)]),
    # a call on the last base of an M op followed by a deletion keeps the
    # pre-deletion offset (the >= of 663)
    ("boundary_del", dict(seq="AAACGA", cigar="3M1D3M", mm="C+m?,0;", ml=[200], pos=700), [(703, 0)]),
    # the walk stops at N: the read is kept with no calls (get_mod_poss_on_ref
    # returns 1 once it has a call and a CIGAR, 771-775)
    ("stop_at_n", dict(seq="AAAACG", cigar="3M100N3M", mm="C+m?,0;", ml=[200], pos=800), []),
    # dropped records
    ("secondary", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0,0;", ml=[200, 10], pos=100, flag=256), None),
    ("supplementary", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0,0;", ml=[200, 10], pos=100, flag=2048), None),
    ("unmapped", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0,0;", ml=[200, 10], pos=100, flag=4), None),
    ("low_mapq", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0,0;", ml=[200, 10], pos=100, mapq=5), None),
    ("high_de", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0,0;", ml=[200, 10], pos=100, de=0.2), None),
    ("no_de_tag", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0,0;", ml=[200, 10], pos=100, de=-1.0),
     [(101, 0), (105, 1)]),
    ("short", dict(seq="ACGT", cigar="4M", mm="C+m?,0;", ml=[200], pos=100), None),
    ("no_mm", dict(seq="ACGTTCGA", cigar="8M", pos=100), None),
    ("only_non_cpg", dict(seq="ACATTCTA", cigar="8M", mm="C+m?,0;", ml=[200], pos=100), None),
    ("call_at_read_end", dict(seq="AATTTTGC", cigar="8M", mm="C+m?,0;", ml=[200], pos=100), None),
    ("skip_past_end", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0,5;", ml=[200, 10], pos=100), None),
    ("ml_too_short", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0,0;", ml=[200], pos=100), None),
    ("malformed_mm", dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0,,1;", ml=[200, 10, 3], pos=100), None),
    ("no_cigar", dict(seq="ACGTTCGA", cigar="", mm="C+m?,0,0;", ml=[200, 10], pos=100), None),
]

LOAD_CFG_SMALL = LoadConfig(min_mapq=10, min_len=6, qual_lo=100, qual_hi=156)


def handmade_batch():
    return records_batch([(0, 10, [r for _, r, _ in HANDMADE])])


def synth_aln(n, cov, seed, **kw):
    return make_aln_batch(AlnSpec(n_windows=n, coverage=cov, seed=seed, **kw))


def aln_cases():
    """(name, batch) record-level parity cases at sizes the oracle finishes in seconds."""
    return [
        ("aln30", synth_aln(4, 30, 41)),
        ("aln_mix_implicit", synth_aln(3, 30, 42, mm_mix=True, implicit_frac=0.3, clip_frac=0.6)),
        ("aln_noisy", synth_aln(3, 30, 43, indel_rate=0.03, sub_rate=0.03, clip_frac=0.5, filt_frac=0.1)),
        ("aln_dense_cpg", synth_aln(2, 30, 44, cpg_rate=0.12, len_scale=0.5)),
        ("aln60", synth_aln(2, 60, 45)),
    ]


def mm_fuzz_batch(seed=17, n=160):
    """Records whose MM/ML texts stress K0's tag parser: several entries
    (h / ChEBI / m / combined codes, '.'/'?' or neither, a missing final ';'),
    texts of 1-6 KB (entries and headers across the parser's 256-byte rows),
    leading zeros, 8-9 digit counts (the SWAR fallback), bytes after the last
    count, and malformed lists (an empty count, a stray byte before the last
    comma, a trailing comma, ML too short).  Every record is CpG-rich so most
    are kept; expected calls come from the oracle."""
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(n):
        L = int(rng.integers(300, 9000))
        # CpG-rich: a third of the positions start a CG
        b = rng.choice(list("ACGT"), L)
        cg = rng.random(L - 1) < 0.08
        b[:-1][cg] = "C"
        b[1:][cg] = "G"
        seq = "".join(b)
        rev = bool(rng.random() < 0.5)
        tgt = "G" if rev else "C"
        n_t = seq.count(tgt)
        # skip list over the read's target bases (original orientation)
        keep = np.flatnonzero(rng.random(n_t) < rng.uniform(0.05, 0.9))
        d = np.diff(np.concatenate([[-1], keep])) - 1
        skips = [str(x) for x in d.tolist()]
        kind = rng.integers(0, 12)
        if kind == 0 and skips:
            skips[0] = "0" * int(rng.integers(1, 4)) + skips[0]              # leading zeros
        if kind == 1 and skips:
            skips[-1] = str(int(rng.integers(10_000_000, 999_999_999)))     # 8-9 digits (past the read)
        if kind == 2 and len(skips) > 1:
            skips[int(rng.integers(0, len(skips)))] = str(int(rng.integers(10_000_000, 99_999_999)))
        lst = ",".join(skips)
        tail = ""
        if kind == 3:
            tail = "x7"                                                      # bytes after the last count
        if kind == 4 and len(skips) > 2:
            j = lst.index(",", 1)
            lst = lst[:j] + "x" + lst[j:]                                    # stray byte before a comma
        if kind == 5 and len(skips) > 2:
            j = lst.index(",", 1)
            lst = lst[:j] + "," + lst[j:]                                    # an empty count
        if kind == 6:
            tail = ","                                                       # trailing comma
        nd = len(skips)
        pre, ml = "", []
        hdr = "C+m" + ["?", ".", ""][int(rng.integers(0, 3))]
        ncm = 1
        lay = int(rng.integers(0, 4))
        if lay == 1:                                                         # h entry first (dorado)
            hl = ",".join(str(x) for x in rng.integers(0, 5, int(rng.integers(1, 900))))
            pre = f"C+h?,{hl};"
            ml += rng.integers(0, 256, hl.count(",") + 1).tolist()
        elif lay == 2:                                                       # ChEBI code first
            cl = ",".join(str(x) for x in rng.integers(0, 30, int(rng.integers(1, 300))))
            pre = f"C+76792?,{cl};"
            ml += rng.integers(0, 256, cl.count(",") + 1).tolist()
        elif lay == 3:                                                       # combined codes
            hdr = "C+hm?"
            ncm = 2
        end = "" if rng.random() < 0.1 else ";"
        post = "" if rng.random() < 0.7 else "A+a?,1,2;"
        mm = f"{pre}{hdr},{lst}{tail}{end}" + (post if end else "")
        ml += rng.integers(0, 256, nd * ncm).tolist()
        if kind == 7 and ml:
            ml = ml[:-1]                                                     # ML too short
        if kind == 8:
            ml = []                                                          # no ML: 255 everywhere
        if post and end:
            ml += [1, 2]
        recs.append(dict(seq=seq, cigar=f"{L}M", mm=mm, ml=ml, pos=10_000 + 20_000 * i, flag=16 if rev else 0))
    return records_batch([(0, 10_000 + 20_000 * n, recs)])

"""Parity-test inputs: seeded synthetic batches plus edge cases of the
reference's window semantics (blockjoin.c line numbers in each docstring)."""
import numpy as np

from pomfret_amd.abi import Config, WindowBatch
from pomfret_amd.synth import SynthSpec, make_batch


def synth(n, cov, seed, **kw):
    return make_batch(SynthSpec(n_windows=n, coverage=cov, seed=seed, **kw))


def report_like(n=3, seed=9):
    """Config 5: `pomfret report --chunk-size 10000 --chunk-stride 5000` at 200x:
    10 kb windows, parameters c/10+1, 2x, c/4+1 (blockjoin.c:5045-5051)."""
    b = synth(n, 200, seed, gap=10_000, window_stride=400_000)
    return b, Config.from_coverage(200, report=True)


def with_odd_tags(b: WindowBatch, seed=3):
    """Left/right reference reads with hp 254 and 7: the (readID<<2)|hp round
    trip of haplotag_region1 step 1.5 (blockjoin.c:4013-4024) moves their tag
    to readID|63 (resp. readID|1)."""
    b = b.select(range(b.n_windows))
    rng = np.random.default_rng(seed)
    sel = rng.random(b.n_reads) < 0.08
    b.read_hp[sel] = rng.choice(np.array([254, 7, 5, 2], np.uint8), sel.sum())
    return b


def with_unsorted_and_dup_calls(b: WindowBatch, seed=4):
    """Some reads get a duplicated call position (another category) and a
    swapped pair of calls: the reference takes first/last calls in array order
    (blockjoin.c:3375-3379) and radix-sorts the rest (:3400)."""
    b = b.select(range(b.n_windows))
    rng = np.random.default_rng(seed)
    pos, cat = list(b.call_pos), list(b.call_cat)
    off = b.read_call_off.astype(np.int64)
    new_pos, new_cat, new_off = [], [], [0]
    for r in range(b.n_reads):
        p = pos[off[r]:off[r + 1]]
        c = cat[off[r]:off[r + 1]]
        if len(p) > 6 and rng.random() < 0.15:
            i = int(rng.integers(1, len(p) - 2))
            p = p[:i] + [p[i]] + p[i:]                # duplicated position
            c = c[:i] + [int((c[i] + 1) % 3)] + c[i:]
        if len(p) > 6 and rng.random() < 0.10:
            i = int(rng.integers(1, len(p) - 2))
            p[i], p[i + 1] = p[i + 1], p[i]           # locally unsorted
            c[i], c[i + 1] = c[i + 1], c[i]
        new_pos += p
        new_cat += c
        new_off.append(len(new_pos))
    return WindowBatch(win_start=b.win_start, win_end=b.win_end, win_read_off=b.win_read_off,
                       read_start=b.read_start, read_end=b.read_end, read_hp=b.read_hp,
                       read_call_off=np.array(new_off, np.uint64),
                       call_pos=np.array(new_pos, np.uint32), call_cat=np.array(new_cat, np.uint8))


def with_empty_and_starved_windows(b: WindowBatch):
    """Window 0 keeps only its first read (left-coverage check fails,
    blockjoin.c:1161); window 1 loses all reads (empty fetch)."""
    keep = []
    ro = b.win_read_off
    for w in range(b.n_windows):
        rs = list(range(ro[w], ro[w + 1]))
        if w == 0:
            rs = rs[:1]
        elif w == 1:
            rs = []
        keep.append(rs)
    reads = np.array([r for rs in keep for r in rs], np.int64)
    co = b.read_call_off.astype(np.int64)
    calls = np.concatenate([np.arange(co[r], co[r + 1]) for r in reads]) if len(reads) else np.zeros(0, np.int64)
    return WindowBatch(
        win_start=b.win_start, win_end=b.win_end,
        win_read_off=np.concatenate([[0], np.cumsum([len(x) for x in keep])]),
        read_start=b.read_start[reads], read_end=b.read_end[reads], read_hp=b.read_hp[reads],
        read_call_off=np.concatenate([[0], np.cumsum(co[reads + 1] - co[reads])]),
        call_pos=b.call_pos[calls], call_cat=b.call_cat[calls])


def handmade():
    """Four sites carried by two reads (see tests/test_oracle.py)."""
    reads = []
    for i in range(30):
        reads.append((10, 60, i % 2, [(50, 0)]))
    reads.append((90, 500, 254, [(100, 0), (200, 1), (300, 0), (400, 1)]))
    reads.append((90, 500, 254, [(100, 1), (200, 0), (300, 1), (400, 0)]))
    off = np.cumsum([0] + [len(r[3]) for r in reads])
    return WindowBatch(
        win_start=[60], win_end=[70], win_read_off=[0, len(reads)],
        read_start=[r[0] for r in reads], read_end=[r[1] for r in reads],
        read_hp=[r[2] for r in reads], read_call_off=off,
        call_pos=[c[0] for r in reads for c in r[3]], call_cat=[c[1] for r in reads for c in r[3]])


def cases():
    """(name, cfg, batch) parity cases at sizes the oracle finishes in seconds."""
    c30 = Config.from_coverage(30, given=False)
    c60 = Config.from_coverage(60, given=True)
    out = [
        ("synth30", c30, synth(12, 30, 21)),
        ("synth60", c60, synth(6, 60, 22)),
        ("gapmix", c30, synth(8, 30, 23, gap_mix=True)),
        ("report200", *reversed(report_like())),
        ("oddtags", c30, with_odd_tags(synth(6, 30, 24))),
        ("unsorted_dups", c30, with_unsorted_and_dup_calls(synth(6, 30, 25))),
        ("starved", c30, with_empty_and_starved_windows(synth(4, 30, 26))),
        ("k1", Config(k=1, k_span=5000, cov_for_selection=4, cov_for_runtime=8, n_cand=8), synth(4, 30, 27)),
        ("k2_span300", Config(k=2, k_span=300, cov_for_selection=4, cov_for_runtime=8, n_cand=8), synth(4, 30, 28)),
        ("k4", Config(k=4, k_span=5000, cov_for_selection=4, cov_for_runtime=8, n_cand=8), synth(4, 30, 29)),
        ("ncand2", Config(k=3, k_span=5000, cov_for_selection=4, cov_for_runtime=8, n_cand=2), synth(4, 30, 30)),
        ("ncand100", Config(k=3, k_span=5000, cov_for_selection=4, cov_for_runtime=8, n_cand=100), synth(3, 30, 31)),
        ("cov_sel_high", Config(k=3, k_span=5000, cov_for_selection=12, cov_for_runtime=30, n_cand=8), synth(4, 30, 32)),
        ("handmade", Config(k=3, k_span=5000, cov_for_selection=1, cov_for_runtime=2, n_cand=4), handmade()),
    ]
    return out


def _batch_from_reads(s, e, reads):
    """One window [s, e] from [(start, end, hp, [(pos, cat), ...]), ...]."""
    off = np.cumsum([0] + [len(r[3]) for r in reads])
    return WindowBatch(
        win_start=[s], win_end=[e], win_read_off=[0, len(reads)],
        read_start=[r[0] for r in reads], read_end=[r[1] for r in reads],
        read_hp=[r[2] for r in reads], read_call_off=off,
        call_pos=[c[0] for r in reads for c in r[3]], call_cat=[c[1] for r in reads for c in r[3]])


# T8 positions and their (meth, unmeth) call counts; the reference's per-site
# counters are u16 with the count in the top 12 bits (cnt += 1<<4,
# blockjoin.c:3210-3238), so a count is n mod 4096.
T8_COUNTS = {100_100: (4100, 20),     # meth wraps to 4  < cov_sel 5: not a site
             100_200: (4101, 20),     # meth wraps to 5 >= 5: a site
             100_300: (4096, 20),     # meth wraps to 0: not a site
             100_400: (20, 20),       # ordinary site
             100_500: (10, 4096)}     # unmeth wraps to 0: not a site
T8_SITES = [100_200, 100_400]         # worked by hand from the rule above
T8_CFG = Config(k=3, k_span=5000, cov_for_selection=5, cov_for_runtime=10, n_cand=8)


def t8_counter_wrap():
    """A window of 4,200 reads, all left-side references (start <= s, hp
    alternating 0/1, so the left-coverage check passes), whose calls give
    every T8 position the counts of T8_COUNTS (read i makes a meth call at
    a position while i < n_meth, an unmeth call while i < n_meth + n_unmeth)."""
    n = 4200
    reads = []
    for i in range(n):
        calls = []
        for p, (nm, nu) in T8_COUNTS.items():
            if i < nm:
                calls.append((p, 0))
            elif i < nm + nu:
                calls.append((p, 1))
        reads.append((50_000, 200_000, i % 2, calls))
    return _batch_from_reads(100_000, 150_000, reads)


def t6_range_wrap():
    """Every site lies right of the gap end e.  Direction 1 starts with
    mmr_min_i = n-1 and decrements it once per site > e
    (haplotag_region1, blockjoin.c:3999-4003): past site 0 the u32 wraps to
    UINT32_MAX, the range update's `int i = mmr_min_i` loop never runs
    (3671) and no site is ever inside [mmr_min_i, mmr_max_i), so direction 1
    tags no read and its join is -1; direction 0 (range from 0 upwards) tags
    normally.  A clamped (non-wrapping) min_i would let direction 1 query
    sites and tag reads."""
    rng = np.random.default_rng(61)
    s, e = 100_000, 150_000
    sites = np.arange(160_000, 190_000, 400)
    meth = rng.random(sites.shape[0]) < 0.5        # allele-specific: hap 0 meth at `meth` sites
    reads = []
    for i in range(40):                            # left references, hp 0/1
        h = i % 2
        reads.append((60_000, 195_000, h, [(int(p), int(meth[k] ^ h)) for k, p in enumerate(sites)]))
    for i in range(40):                            # untagged reads inside the gap, spanning the sites
        h = int(rng.integers(0, 2))
        reads.append((110_000 + 500 * i, 196_000, 254, [(int(p), int(meth[k] ^ h)) for k, p in enumerate(sites)]))
    for i in range(30):                            # right references (start > s, end >= e), hp 0/1
        h = i % 2
        reads.append((120_000 + 700 * i, 198_000, h, [(int(p), int(meth[k] ^ h)) for k, p in enumerate(sites)]))
    return _batch_from_reads(s, e, reads)


# ---------------------------------------------------------------------------
# -u pre-pass edge cases (reference blockjoin.c:1545-1840) for the wave kernel:
# MD strings the serial machine treats specially, CIGARs with many ops, known
# tables with same-position runs.
def _rand_md(rng, n_tok):
    """MD-like string: numbers (some with leading zeros / many digits),
    mismatch letters (runs of 1-3), '^' runs of 1-150 letters, some holding a
    second '^' (absorbed into the run, :1641-1652), and lowercase / N / U."""
    letters = np.frombuffer(b"ACGTNUacgtnu", np.uint8)
    out = []
    kind = int(rng.integers(0, 3))          # first token: number, letter or '^'
    for _ in range(n_tok):
        if kind == 0:
            v = int(rng.integers(0, 400)) if rng.random() < 0.9 else int(rng.integers(0, 10 ** 6))
            s = str(v)
            if rng.random() < 0.05:
                s = "0" * int(rng.integers(1, 4)) + s
            out.append(s)
            kind = int(rng.integers(1, 3))
        elif kind == 1:
            n = int(rng.integers(1, 4))
            out.append(bytes(letters[rng.integers(0, 12, n)]).decode())
            kind = 0 if rng.random() < 0.8 else int(rng.integers(1, 3))
        else:
            n = int(rng.integers(1, 150)) if rng.random() < 0.2 else int(rng.integers(1, 4))
            body = bytearray(letters[rng.integers(0, 12, n)])
            if rng.random() < 0.1 and n > 1:
                body[int(rng.integers(1, n))] = ord("^")
            out.append("^" + body.decode())
            kind = 0 if rng.random() < 0.9 else 1
    return "".join(out)


def u_quirks(seed=5, n_reads=300):
    """make_u_batch reads with a third of the MD strings replaced by _rand_md,
    a sixth of the CIGARs split into many short M/I/N/H/P ops (>64 ops), and
    extra known entries making 2- and 3-long runs at one position."""
    from pomfret_amd.abi import KnownVars, ReadAlnBatch
    from pomfret_amd.synth_u import USpec, make_u_batch
    known, reads, _ = make_u_batch(USpec(n_reads=n_reads, ref_len=200_000, mean_len=6000,
                                         var_every=200, indel_frac=0.3, seed=seed))
    rng = np.random.default_rng(seed)
    # known: duplicate ~15% of the entries (one or two extra copies at the same
    # position, alternating haptag and chars), keeping VCF order
    kp, kl, ko, kh, kc, koff = [], [], [], [], [], [0]
    for i in range(len(known.pos)):
        reps = 1 + (int(rng.integers(1, 3)) if rng.random() < 0.15 else 0)
        for c in range(reps):
            kp.append(int(known.pos[i])); kl.append(int(known.len[i])); ko.append(int(known.op[i]))
            kh.append(int(known.haptag[i]) ^ (c & 1))
            ch = known.chars[known.char_off[i]:known.char_off[i + 1]].tolist()
            if c:
                ch = [(x + c) % 4 for x in ch]
            kc += ch
            koff.append(len(kc))
    known = KnownVars(pos=np.array(kp), len=np.array(kl), op=np.array(ko), haptag=np.array(kh),
                      char_off=np.array(koff), chars=np.array(kc, np.uint8))
    cig, cig_off, md, md_off = [], [0], [], [0]
    for r in range(reads.n_reads):
        c = reads.cigar[reads.cigar_off[r]:reads.cigar_off[r + 1]].tolist()
        m = bytes(reads.md[reads.md_off[r]:reads.md_off[r + 1]])
        u = rng.random()
        if u < 0.33:
            m = _rand_md(rng, int(rng.integers(1, 400))).encode()
        elif u < 0.5:
            nc = []
            for w in c:
                op, ln = w & 0xf, w >> 4
                if op == 0 and ln > 8:
                    while ln > 0:
                        k = min(ln, int(rng.integers(1, 6)))
                        nc.append(k << 4 | 0)
                        ln -= k
                        x = rng.random()
                        if x < 0.3:
                            nc.append(int(rng.integers(1, 4)) << 4 | 1)
                        elif x < 0.35:
                            nc.append(int(rng.integers(1, 3)) << 4 | int(rng.choice([3, 5, 6])))
                else:
                    nc.append(w)
            c = nc
        cig += c
        cig_off.append(len(cig))
        md.append(np.frombuffer(m, np.uint8))
        md_off.append(md_off[-1] + len(m))
    reads = ReadAlnBatch(start=reads.start, end=reads.end, cigar_off=np.array(cig_off),
                         cigar=np.array(cig, np.uint32), seq_off=reads.seq_off, seq_len=reads.seq_len,
                         seq=reads.seq, md_off=np.array(md_off), md=np.concatenate(md))
    return known, reads

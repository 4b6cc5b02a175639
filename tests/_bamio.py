"""Test-side BAM + BAI writer (SAM/BAM specification, SAMv1 4.1-4.2, 5.2),
independent of the library's reader: BGZF blocks by zlib raw deflate, the
index's bins / chunks / 16 kb linear index / metadata pseudo-bin built as
htslib's indexer does.  Used to make BAM fixtures for tests/test_bam.py;
test infrastructure, never imported by the product."""
from __future__ import annotations

import struct
import zlib
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

BLOCK = 0xFF00          # htslib BGZF_BLOCK_SIZE: uncompressed bytes per block
EOF_BLOCK = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def reg2bin(beg: int, end: int) -> int:
    end -= 1
    if beg >> 14 == end >> 14:
        return ((1 << 15) - 1) // 7 + (beg >> 14)
    if beg >> 17 == end >> 17:
        return ((1 << 12) - 1) // 7 + (beg >> 17)
    if beg >> 20 == end >> 20:
        return ((1 << 9) - 1) // 7 + (beg >> 20)
    if beg >> 23 == end >> 23:
        return ((1 << 6) - 1) // 7 + (beg >> 23)
    if beg >> 26 == end >> 26:
        return ((1 << 3) - 1) // 7 + (beg >> 26)
    return 0


def ref_len(cigar) -> int:
    return int(sum(c >> 4 for c in cigar if (c & 15) in (0, 2, 3, 7, 8)))


def endpos(pos: int, cigar, flag: int) -> int:
    rl = 0 if (flag & 4) else ref_len(cigar)
    return pos + (rl if rl > 0 else 1)


@dataclass
class Rec:
    tid: int
    pos: int
    qname: str
    flag: int = 0
    mapq: int = 60
    cigar: List[int] = field(default_factory=list)    # BAM encoding len<<4|op
    seq: bytes = b""                                  # 4-bit packed, (l+1)//2 bytes
    l_seq: int = 0
    aux: bytes = b""
    bin_override: Optional[int] = None
    qual: Optional[bytes] = None                      # None: absent (0xFF)


def aux_Z(tag: str, s: str) -> bytes:
    return tag.encode() + b"Z" + s.encode() + b"\0"


def aux_i(tag: str, v: int) -> bytes:
    return tag.encode() + b"i" + struct.pack("<i", v)


def aux_C(tag: str, v: int) -> bytes:
    return tag.encode() + b"C" + struct.pack("<B", v)


def aux_f(tag: str, v: float) -> bytes:
    return tag.encode() + b"f" + struct.pack("<f", v)


def aux_BC(tag: str, vals) -> bytes:
    vals = bytes(bytearray(vals))
    return tag.encode() + b"BC" + struct.pack("<I", len(vals)) + vals


def aux_BI(tag: str, vals) -> bytes:
    vals = list(vals)
    return tag.encode() + b"BI" + struct.pack("<I", len(vals)) + struct.pack(f"<{len(vals)}I", *vals)


def encode_record(r: Rec) -> bytes:
    qn = r.qname.encode() + b"\0"
    end = endpos(r.pos, r.cigar, r.flag) if r.pos >= 0 else 0
    b = r.bin_override if r.bin_override is not None else (reg2bin(r.pos, end) if r.pos >= 0 else 4680)
    body = struct.pack("<iiBBHHHiiii", r.tid, r.pos, len(qn), r.mapq, b, len(r.cigar), r.flag, r.l_seq,
                       -1, -1, 0)
    ql = r.qual if r.qual is not None else b"\xff" * r.l_seq
    body += qn + struct.pack(f"<{len(r.cigar)}I", *r.cigar) + bytes(r.seq) + ql + r.aux
    return struct.pack("<i", len(body)) + body


class _Bgzf:
    """BGZF writer tracking virtual offsets as htslib's bgzf_write does (a
    full block is flushed at once, so an offset never points at a block's
    end)."""

    def __init__(self):
        self.out = bytearray()
        self.buf = bytearray()

    def tell(self) -> int:
        return (len(self.out) << 16) | len(self.buf)

    def _flush(self):
        if not self.buf:
            return
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        data = c.compress(bytes(self.buf)) + c.flush()
        bsize = 18 + len(data) + 8
        hdr = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize - 1)
        self.out += hdr + data + struct.pack("<II", zlib.crc32(bytes(self.buf)) & 0xFFFFFFFF, len(self.buf))
        self.buf = bytearray()

    def write(self, data: bytes):
        i = 0
        while i < len(data):
            k = min(BLOCK - len(self.buf), len(data) - i)
            self.buf += data[i:i + k]
            i += k
            if len(self.buf) == BLOCK:
                self._flush()

    def flush(self):
        self._flush()

    def close(self) -> bytes:
        self._flush()
        return bytes(self.out) + EOF_BLOCK


def _deflate_block(args):
    data, level = args
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    z = c.compress(data) + c.flush()
    bsize = 18 + len(z) + 8
    hdr = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize - 1)
    return hdr + z + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))


class _BgzfPar:
    """The same block boundaries as _Bgzf, blocks compressed at close() in a
    process pool; tell() returns a token (raw block index << 16 | offset) that
    translate() turns into the virtual offset once block addresses are known."""

    def __init__(self, level: int, workers: int):
        self.level, self.workers = level, workers
        self.blocks = []
        self.buf = bytearray()
        self.addr = None

    def tell(self) -> int:
        return (len(self.blocks) << 16) | len(self.buf)

    def _flush(self):
        if self.buf:
            self.blocks.append(bytes(self.buf))
            self.buf = bytearray()

    def write(self, data: bytes):
        i = 0
        while i < len(data):
            k = min(BLOCK - len(self.buf), len(data) - i)
            self.buf += data[i:i + k]
            i += k
            if len(self.buf) == BLOCK:
                self._flush()

    def flush(self):
        self._flush()

    def close(self) -> bytes:
        self._flush()
        import multiprocessing as mp
        with mp.get_context("fork").Pool(self.workers) as pool:
            comp = pool.map(_deflate_block, [(b, self.level) for b in self.blocks], chunksize=16)
        self.addr = np.concatenate([[0], np.cumsum([len(c) for c in comp])]).astype(np.int64)
        return b"".join(comp) + EOF_BLOCK

    def translate(self, tok: int) -> int:
        return (int(self.addr[tok >> 16]) << 16) | (tok & 0xFFFF)


def bam_header(refs, text: str = "@HD\tVN:1.6\tSO:coordinate\n") -> bytes:
    hdr = b"BAM\1" + struct.pack("<i", len(text)) + text.encode() + struct.pack("<i", len(refs))
    for name, ln in refs:
        nb = name.encode() + b"\0"
        hdr += struct.pack("<i", len(nb)) + nb + struct.pack("<i", ln)
    return hdr


def bai_bytes(nref: int, entries) -> bytes:
    """The BAI of records given in file order as (tid, pos, end, flag, u, v)
    (virtual offsets of each record's start and end; tid < 0: unplaced), the
    way htslib's indexer builds it: bins with contiguous chunks merged, the
    16 kb linear index with gaps filled by the previous offset, the metadata
    pseudo-bin, n_no_coor."""
    bins = [dict() for _ in range(nref)]       # bin -> [[u, v], ...]
    lin = [dict() for _ in range(nref)]
    meta = [[None, None, 0, 0] for _ in range(nref)]
    last_bin = [None] * nref
    n_no_coor = 0
    for t, pos, end, flag, u, v in entries:
        if t < 0:
            n_no_coor += 1
            continue
        b = reg2bin(pos, end)
        ch = bins[t].setdefault(b, [])
        if last_bin[t] == b and ch and ch[-1][1] == u:
            ch[-1][1] = v                      # contiguous records of one bin: one chunk
        else:
            ch.append([u, v])
        last_bin[t] = b
        for wdw in range(pos >> 14, ((end - 1) >> 14) + 1):
            lin[t].setdefault(wdw, u)
        m = meta[t]
        if m[0] is None:
            m[0] = u
        m[1] = v
        if flag & 4:
            m[3] += 1
        else:
            m[2] += 1
    idx = bytearray(b"BAI\1" + struct.pack("<i", nref))
    for t in range(nref):
        bl = sorted(bins[t].items())
        has_meta = meta[t][0] is not None
        idx += struct.pack("<i", len(bl) + (1 if has_meta else 0))
        for b, chunks in bl:
            idx += struct.pack("<Ii", b, len(chunks))
            for u, v in chunks:
                idx += struct.pack("<QQ", u, v)
        if has_meta:
            idx += struct.pack("<Ii", 37450, 2) + struct.pack("<QQQQ", meta[t][0], meta[t][1], meta[t][2], meta[t][3])
        n_intv = (max(lin[t]) + 1) if lin[t] else 0
        idx += struct.pack("<i", n_intv)
        prev = 0
        for wdw in range(n_intv):
            val = lin[t].get(wdw, prev)        # htslib fills a gap with the previous offset
            idx += struct.pack("<Q", val)
            prev = val
    idx += struct.pack("<Q", n_no_coor)
    return bytes(idx)


def write_bam(path: str, refs, recs: List[Rec], bai_path: Optional[str] = None, text: str = "@HD\tVN:1.6\tSO:coordinate\n",
              workers: int = 0, level: int = 6):
    """refs: [(name, length)]; recs sorted by (tid, pos) with unplaced reads
    (tid -1) last.  Writes path and path + '.bai' (or bai_path).  workers > 1
    compresses the blocks in a process pool (same bytes as the serial writer
    at the same level)."""
    z = _BgzfPar(level, workers) if workers > 1 else _Bgzf()
    z.write(bam_header(refs, text))
    z.flush()                                  # bam_hdr_write flushes the header block
    entries = []
    for r in recs:
        u = z.tell()
        z.write(encode_record(r))
        v = z.tell()
        end = endpos(r.pos, r.cigar, r.flag) if r.tid >= 0 else 0
        entries.append((r.tid, r.pos, end, r.flag, u, v))
    data = z.close()
    if workers > 1:                            # tokens -> virtual offsets
        tr = z.translate
        entries = [(t, p, e, f, tr(u), tr(v)) for t, p, e, f, u, v in entries]
    with open(path, "wb") as f:
        f.write(data)
    with open(bai_path or path + ".bai", "wb") as f:
        f.write(bai_bytes(len(refs), entries))


def records_from_aln(aln, tid: int = 0, prefix: str = "r", hp_zero_every: int = 0, de_absent_every: int = 0,
                     qual: bool = False, seed: int = 0):
    """One Rec per record of an AlnBatch (tests/_aln_cases / synth_aln), with
    MM:Z, ML:B:C, MD:Z (when the generator made one), HP:i (absent for 254; HP:i:0 every hp_zero_every-th
    unphased record) and de:f (absent when < 0).  qual=True gives every record
    a QUAL string (slices of a pool of Phred values ~ N(20, 6), nanopore-like
    entropy) instead of the absent 0xFF run, so BGZF sizes and inflate work
    are those of a real BAM."""
    out = []
    pool = None
    if qual:
        rng = np.random.default_rng(seed)
        pool = rng.normal(20, 6, 1 << 24).clip(2, 50).astype(np.uint8).tobytes()
        starts = rng.integers(0, (1 << 24) - 1, aln.n_recs)
    for i in range(aln.n_recs):
        cig = [int(x) for x in aln.cigar[aln.cigar_off[i]:aln.cigar_off[i + 1]]]
        lq = int(aln.l_qseq[i])
        seq = bytes(aln.seq[aln.seq_off[i]:aln.seq_off[i] + (lq + 1) // 2])
        aux = b""
        hp = int(aln.hp[i])
        if hp in (0, 1):
            aux += aux_i("HP", hp + 1)
        elif hp != 254:
            aux += aux_i("HP", hp + 1)
        elif hp_zero_every and i % hp_zero_every == 0:
            aux += aux_C("HP", 0)
        de = float(aln.de[i])
        if de >= 0 and not (de_absent_every and i % de_absent_every == 0):
            aux += aux_f("de", de)
        mm = bytes(aln.mm[aln.mm_off[i]:aln.mm_off[i + 1]]).decode()
        if mm:
            aux += aux_Z("MM", mm)
        ml = aln.ml[aln.ml_off[i]:aln.ml_off[i + 1]]
        if len(ml):
            aux += aux_BC("ML", ml)
        if "md" in aln.meta:
            aux += aux_Z("MD", aln.meta["md"][i])
        q = None
        if pool is not None:
            o = int(starts[i]) % max(1, (1 << 24) - lq)
            q = pool[o:o + lq]
        out.append(Rec(tid=tid, pos=int(aln.pos[i]), qname=f"{prefix}{i}", flag=int(aln.flag[i]),
                       mapq=int(aln.mapq[i]), cigar=cig, seq=seq, l_seq=lq, aux=aux, qual=q))
    return out


def expected_fetch(recs: List[Rec], tid: int, s: int, e: int, readback: int) -> List[int]:
    """Indices of recs that load_reads_given_interval's region query returns,
    by the overlap rule alone (no index): region chrom:b-(e+rb) with
    b = max(s-rb, 0) is the 0-based [max(b-1, 0), e+rb)."""
    b1 = s - readback if s - readback > 0 else 0
    beg, end = (b1 - 1 if b1 > 0 else 0), e + readback
    return [i for i, r in enumerate(recs)
            if r.tid == tid and r.pos < end and endpos(r.pos, r.cigar, r.flag) > beg]


def _vcf_header(contigs):
    return ["##fileformat=VCFv4.2"] + [f"##contig=<ID={c},length={n}>" for c, n in contigs] + [
        '##FORMAT=<ID=GT,Number=1,Type=String,Description="Genotype">',
        '##FORMAT=<ID=PS,Number=1,Type=Integer,Description="Phase set">',
        "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1"]


def phased_vcf_lines(chrom: str, windows):
    """Body lines of write_phased_vcf for one contig."""
    lines = []
    first = max(1, windows[0][0] - 1000)
    ps = first
    pts = [(first, ps)]
    for s, e in windows:
        pts.append((s, ps))
        ps = e
        pts.append((e, ps))
    pts.append((windows[-1][1] + 1000, ps))
    for k, (pos, p) in enumerate(pts):
        gt = "0|1" if k % 2 == 0 else "1|0"
        lines.append(f"{chrom}\t{pos}\t.\tA\tG\t50\tPASS\t.\tGT:PS\t{gt}:{p}")
    return lines


def write_vcf_multi(path: str, contigs, bodies):
    """A multi-contig VCF: header with `contigs` [(name, length)], then the
    body lines of each contig in the order given."""
    with open(path, "w") as f:
        f.write("\n".join(_vcf_header(contigs) + [ln for b in bodies for ln in b]) + "\n")


def write_phased_vcf(path: str, chrom: str, windows, chrom_len: int = 100_000_000):
    """A one-sample phased VCF whose phase-block gaps are exactly `windows`
    [(s, e), ...] (sorted, far apart): block k ends with a variant at POS s_k
    and block k+1 starts at POS e_k with PS e_k (insert_vcf_line's gap is
    [last POS of a block, PS of the next])."""
    lines = ["##fileformat=VCFv4.2", f"##contig=<ID={chrom},length={chrom_len}>",
             '##FORMAT=<ID=GT,Number=1,Type=String,Description="Genotype">',
             '##FORMAT=<ID=PS,Number=1,Type=Integer,Description="Phase set">',
             "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1"]
    first = max(1, windows[0][0] - 1000)
    ps = first
    pts = [(first, ps)]
    for s, e in windows:
        pts.append((s, ps))
        ps = e
        pts.append((e, ps))
    pts.append((windows[-1][1] + 1000, ps))
    for k, (pos, p) in enumerate(pts):
        gt = "0|1" if k % 2 == 0 else "1|0"
        lines.append(f"{chrom}\t{pos}\t.\tA\tG\t50\tPASS\t.\tGT:PS\t{gt}:{p}")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def write_u_vcf(path: str, chrom: str, aln, chrom_len: int = 400_000_000):
    """The phased VCF of a synth_aln batch made with het SNVs: every window's
    SNVs, the left side (POS <= s) in the block that ends at the gap, the
    right side (POS >= e) in the block that starts there with PS e, so
    insert_vcf_line's gaps are exactly the windows.  GT "a|b" puts ALT on the
    block haplotype that carries it: h_alt left of the gap, h_alt ^ orient
    right of it (the generator's HP convention: right-side reads carry
    truth ^ orient)."""
    lines = ["##fileformat=VCFv4.2", f"##contig=<ID={chrom},length={chrom_len}>",
             '##FORMAT=<ID=GT,Number=1,Type=String,Description="Genotype">',
             '##FORMAT=<ID=PS,Number=1,Type=Integer,Description="Phase set">',
             "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1"]
    lines += u_vcf_lines(chrom, aln)
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def u_vcf_lines(chrom: str, aln):
    """Body lines of write_u_vcf for one contig."""
    lines = []
    ps = None
    for w in range(aln.n_windows):
        sv = aln.meta["snv"][w]
        s, e, orient = int(aln.win_start[w]), int(aln.win_end[w]), int(aln.meta["orient"][w])
        for p0, r, a, h in zip(sv["pos"].tolist(), sv["ref"].tolist(), sv["alt"].tolist(), sv["h_alt"].tolist()):
            pos = p0 + 1
            if pos <= s:
                hb = h
                if ps is None:
                    ps = pos
            else:
                hb = h ^ orient
                if pos == e:
                    ps = e
            gt = "0|1" if hb == 1 else "1|0"
            lines.append(f"{chrom}\t{pos}\t.\t{'ACGT'[r]}\t{'ACGT'[a]}\t50\tPASS\t.\tGT:PS\t{gt}:{ps}")
    return lines

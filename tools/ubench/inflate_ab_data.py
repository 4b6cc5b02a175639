"""Test data for inflate_ab: BGZF blocks of BAM-like content (4-bit SEQ +
quality strings) written to argv[1]; two mixes: QUAL-heavy (one 10 kb read
segment per block) and SEQ-heavy.  argv[2] = "huff": Huffman-only streams
(no matches), to separate the literal path from the match path."""
import sys
import zlib
import struct
import numpy as np


def bgzf_block(data: bytes, level: int = 6) -> bytes:
    strat = zlib.Z_HUFFMAN_ONLY if len(sys.argv) > 2 and sys.argv[2] == "huff" else zlib.Z_DEFAULT_STRATEGY
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strat)
    z = c.compress(data) + c.flush()
    bsize = 18 + len(z) + 8
    hdr = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize - 1)
    return hdr + z + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))


rng = np.random.default_rng(3)
out = []
for i in range(32):
    ls = 20000 if i < 16 else 80000
    seq = rng.integers(0, 16, ls, dtype=np.uint8)
    seqb = (seq[0::2] << 4 | seq[1::2]).astype(np.uint8).tobytes()
    q = rng.normal(20, 6, 65536).clip(2, 50).astype(np.uint8).tobytes()
    out.append(bgzf_block((seqb + q)[:65280]))
open(sys.argv[1], "wb").write(b"".join(out))

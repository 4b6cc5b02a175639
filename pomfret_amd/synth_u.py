"""Seeded synthetic input for the --bam-is-untagged (-u) pre-pass
(SURVEY.md 8d): one contig, phased het variants (mostly SNVs, some short
insertions/deletions) and reads sampled from one haplotype with substitution
and indel errors, encoded as BAM-style CIGAR / MD:Z / 4-bit SEQ consistent with
a random reference sequence.

The known-variant table is what insert_variant_from_vcf_line
(reference blockjoin.c:1432-1543) keeps from the phased VCF lines:
  SNV  `X` at POS-1, chars = ALT;   DEL `D` at POS (first deleted base),
  chars = REF[1:];   INS `I` at POS-1 (anchor), chars = ALT[1:];
  haptag = GT[0] (the haplotype carrying REF).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .abi import KnownVars, ReadAlnBatch

BASES = np.frombuffer(b"ACGT", np.uint8)
NIB = {ord("A"): 1, ord("C"): 2, ord("G"): 4, ord("T"): 8}
NT4 = {ord("A"): 0, ord("C"): 1, ord("G"): 2, ord("T"): 3}


@dataclass
class USpec:
    ref_len: int = 400_000
    var_every: int = 1000
    indel_frac: float = 0.12
    n_reads: int = 600
    mean_len: int = 12_000
    sub_err: float = 0.005        # SUP-like; HAC-like: 0.02
    indel_err: float = 0.003      # HAC-like: 0.01
    clip_frac: float = 0.3
    seed: int = 7


def _encode_seq(s: np.ndarray) -> np.ndarray:
    nib = np.zeros(len(s), np.uint8)
    for b, v in NIB.items():
        nib[s == b] = v
    if len(nib) % 2:
        nib = np.concatenate([nib, [0]]).astype(np.uint8)
    return (nib[0::2] << 4 | nib[1::2]).astype(np.uint8)


def make_u_batch(spec: USpec):
    rng = np.random.default_rng(spec.seed)
    ref = BASES[rng.integers(0, 4, spec.ref_len)]
    # --- phased variants (0-based REF position p of the VCF record)
    pos = np.arange(spec.var_every, spec.ref_len - spec.var_every, spec.var_every)
    pos = pos + rng.integers(-spec.var_every // 3, spec.var_every // 3, len(pos))
    kind = np.where(rng.random(len(pos)) < spec.indel_frac, rng.integers(1, 3, len(pos)), 0)
    alt_on = rng.integers(0, 2, len(pos))      # haplotype carrying ALT
    vars_ = []                                 # (p, kind, ref_allele, alt_allele, alt_hap)
    for p, k, h in zip(pos.tolist(), kind.tolist(), alt_on.tolist()):
        r0 = int(ref[p])
        if k == 0:                                         # SNV
            alt = int(BASES[(np.where(BASES == r0)[0][0] + rng.integers(1, 4)) % 4])
            vars_.append((p, 0, bytes([r0]), bytes([alt]), h))
        elif k == 1:                                       # DEL of 1-3 bases after the anchor
            L = int(rng.integers(1, 4))
            vars_.append((p, 1, bytes(ref[p:p + 1 + L]), bytes([r0]), h))
        else:                                              # INS of 1-3 bases after the anchor
            L = int(rng.integers(1, 4))
            ins = bytes(BASES[rng.integers(0, 4, L)])
            vars_.append((p, 2, bytes([r0]), bytes([r0]) + ins, h))
    # known table as the VCF loader stores it
    kp, kl, ko, kh, kc, koff = [], [], [], [], [], [0]
    for p, k, ra, aa, h in vars_:
        gt0 = 1 if h == 0 else 0                           # GT[0] = allele on hap0
        if k == 0:
            kp.append(p); kl.append(1); ko.append(1); chars = aa
        elif k == 1:
            kp.append(p + 1); kl.append(len(ra) - len(aa)); ko.append(3); chars = ra[1:]
        else:
            kp.append(p); kl.append(len(aa) - len(ra)); ko.append(2); chars = aa[1:]
        kh.append(gt0)                                     # haptag = GT[0]
        kc += [NT4[c] for c in chars]
        koff.append(len(kc))
    known = KnownVars(pos=np.array(kp), len=np.array(kl), op=np.array(ko), haptag=np.array(kh),
                      char_off=np.array(koff), chars=np.array(kc, np.uint8))
    var_at = {v[0]: v for v in vars_}

    # --- reads
    starts = np.sort(rng.integers(1000, spec.ref_len - spec.mean_len * 3, spec.n_reads))
    out = dict(start=[], end=[], cig=[], cig_off=[0], seq=[], seq_off=[0], seq_len=[], md=[],
               md_off=[0], hap=[])
    for s in starts.tolist():
        hap = int(rng.integers(0, 2))
        L = int(rng.integers(spec.mean_len // 2, spec.mean_len * 3 // 2))
        cig, seq, md = [], [], []
        match_run = 0
        mrun = 0

        def add_cig(op, n):
            if n <= 0:
                return
            if cig and (cig[-1] & 0xf) == op:
                cig[-1] += n << 4
            else:
                cig.append(n << 4 | op)

        lead = int(rng.integers(1, 200)) if rng.random() < spec.clip_frac else 0
        if lead:
            seq += BASES[rng.integers(0, 4, lead)].tolist()
            add_cig(4, lead)
        p = s
        end_ref = min(s + L, spec.ref_len - 10)
        while p < end_ref:
            v = var_at.get(p)
            if v is not None and v[4] == hap:              # haplotype carries ALT here
                _, k, ra, aa, _ = v
                if k == 0:
                    md.append(str(match_run)); md.append(chr(ra[0])); match_run = 0
                    seq.append(aa[0]); add_cig(0, 1); p += 1
                    continue
                # anchor base matches
                seq.append(int(ref[p])); add_cig(0, 1); match_run += 1; p += 1
                if k == 1:
                    dl = len(ra) - 1
                    md.append(str(match_run)); md.append("^" + ra[1:].decode()); match_run = 0
                    add_cig(2, dl); p += dl
                else:
                    il = len(aa) - 1
                    seq += list(aa[1:]); add_cig(1, il)
                continue
            x = rng.random()
            if x < spec.sub_err:
                b = int(ref[p])
                alt = int(BASES[(np.where(BASES == b)[0][0] + rng.integers(1, 4)) % 4])
                md.append(str(match_run)); md.append(chr(b)); match_run = 0
                seq.append(alt); add_cig(0, 1); p += 1
            elif x < spec.sub_err + spec.indel_err / 2 and cig and (cig[-1] & 0xf) == 0:
                dl = int(rng.integers(1, 3))
                md.append(str(match_run)); md.append("^" + bytes(ref[p:p + dl]).decode()); match_run = 0
                add_cig(2, dl); p += dl
            elif x < spec.sub_err + spec.indel_err and cig and (cig[-1] & 0xf) == 0:
                il = int(rng.integers(1, 3))
                seq += BASES[rng.integers(0, 4, il)].tolist(); add_cig(1, il)
            else:
                seq.append(int(ref[p])); add_cig(0, 1); match_run += 1; p += 1
        md.append(str(match_run))
        if rng.random() < spec.clip_frac:
            tl = int(rng.integers(1, 200))
            seq += BASES[rng.integers(0, 4, tl)].tolist()
            add_cig(4, tl)
        out["start"].append(s)
        out["end"].append(p)
        out["cig"] += cig
        out["cig_off"].append(len(out["cig"]))
        sq = np.array(seq, np.uint8)
        enc = _encode_seq(sq)
        out["seq"].append(enc)
        out["seq_off"].append(out["seq_off"][-1] + len(enc))
        out["seq_len"].append(len(sq))
        mds = "".join(md).encode()
        out["md"].append(np.frombuffer(mds, np.uint8))
        out["md_off"].append(out["md_off"][-1] + len(mds))
        out["hap"].append(hap)
    reads = ReadAlnBatch(
        start=np.array(out["start"]), end=np.array(out["end"]),
        cigar_off=np.array(out["cig_off"]), cigar=np.array(out["cig"], np.uint32),
        seq_off=np.array(out["seq_off"]), seq_len=np.array(out["seq_len"]),
        seq=np.concatenate(out["seq"]), md_off=np.array(out["md_off"]),
        md=np.concatenate(out["md"]))
    return known, reads, np.array(out["hap"], np.uint8)

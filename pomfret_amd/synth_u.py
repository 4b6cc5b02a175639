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


def make_u_batch(spec: USpec, with_vcf: bool = False):
    """known table, reads, true haplotype per read; with_vcf: also the VCF
    records [(POS 1-based, REF, ALT, GT)] the known table is loaded from."""
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

    # --- reads, event-driven: match runs between sparse events (the read's
    # ALT alleles and sequencing errors) are copied from the reference slab
    var_pos = np.array(sorted(var_at), np.int64)
    starts = np.sort(rng.integers(1000, spec.ref_len - spec.mean_len * 3, spec.n_reads))
    out = dict(start=[], end=[], cig=[], cig_off=[0], seq=[], seq_off=[0], seq_len=[], md=[],
               md_off=[0], hap=[])
    p_err = spec.sub_err + spec.indel_err
    for s in starts.tolist():
        hap = int(rng.integers(0, 2))
        L = int(rng.integers(spec.mean_len // 2, spec.mean_len * 3 // 2))
        end_ref = min(s + L, spec.ref_len - 10)
        cig, seq_parts, md = [], [], []

        def add_cig(op, n):
            if n <= 0:
                return
            if cig and (cig[-1] & 0xf) == op:
                cig[-1] += n << 4
            else:
                cig.append(n << 4 | op)

        lead = int(rng.integers(1, 200)) if rng.random() < spec.clip_frac else 0
        if lead:
            seq_parts.append(BASES[rng.integers(0, 4, lead)])
            add_cig(4, lead)
        # events in [s, end_ref): (pos, kind) kind 0 = variant, 1 = error
        vlo, vhi = np.searchsorted(var_pos, [s, end_ref])
        evs = [(int(q), 0) for q in var_pos[vlo:vhi] if var_at[int(q)][4] == hap]
        n_span = end_ref - s
        eq = np.nonzero(rng.random(n_span) < p_err)[0] + s
        evs += [(int(q), 1) for q in eq]
        evs.sort()
        p = s
        match_run = 0
        last_op_m = False            # indel errors only right after a match
        for q, kind in evs:
            if q < p:
                continue
            if q > p:                 # match run up to the event
                seq_parts.append(ref[p:q])
                add_cig(0, q - p)
                match_run += q - p
                p = q
                last_op_m = True
            if kind == 0:
                _, k, ra, aa, _ = var_at[q]
                if k == 0:
                    md.append(str(match_run)); md.append(chr(ra[0])); match_run = 0
                    seq_parts.append(np.array([aa[0]], np.uint8)); add_cig(0, 1); p += 1
                else:
                    seq_parts.append(ref[p:p + 1]); add_cig(0, 1); match_run += 1; p += 1
                    if k == 1:
                        dl = len(ra) - 1
                        md.append(str(match_run)); md.append("^" + ra[1:].decode()); match_run = 0
                        add_cig(2, dl); p += dl
                    else:
                        seq_parts.append(np.frombuffer(aa[1:], np.uint8)); add_cig(1, len(aa) - 1)
                last_op_m = k != 1 and k != 2
                continue
            x = rng.random() * p_err
            if x < spec.sub_err or not last_op_m:
                b = int(ref[p])
                alt = int(BASES[(np.where(BASES == b)[0][0] + rng.integers(1, 4)) % 4])
                md.append(str(match_run)); md.append(chr(b)); match_run = 0
                seq_parts.append(np.array([alt], np.uint8)); add_cig(0, 1); p += 1
                last_op_m = True
            elif x < spec.sub_err + spec.indel_err / 2:
                dl = int(rng.integers(1, 3))
                md.append(str(match_run)); md.append("^" + bytes(ref[p:p + dl]).decode()); match_run = 0
                add_cig(2, dl); p += dl
                last_op_m = False
            else:
                il = int(rng.integers(1, 3))
                seq_parts.append(BASES[rng.integers(0, 4, il)]); add_cig(1, il)
                last_op_m = False
        if p < end_ref:
            seq_parts.append(ref[p:end_ref])
            add_cig(0, end_ref - p)
            match_run += end_ref - p
            p = end_ref
        md.append(str(match_run))
        if rng.random() < spec.clip_frac:
            tl = int(rng.integers(1, 200))
            seq_parts.append(BASES[rng.integers(0, 4, tl)])
            add_cig(4, tl)
        out["start"].append(s)
        out["end"].append(p)
        out["cig"] += cig
        out["cig_off"].append(len(out["cig"]))
        sq = np.concatenate(seq_parts).astype(np.uint8) if seq_parts else np.zeros(0, np.uint8)
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
    if with_vcf:
        recs = [(p + 1, ra.decode(), aa.decode(), f"{1 if h == 0 else 0}|{0 if h == 0 else 1}")
                for p, k, ra, aa, h in vars_]
        return known, reads, np.array(out["hap"], np.uint8), recs
    return known, reads, np.array(out["hap"], np.uint8)

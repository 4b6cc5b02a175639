"""`pomfret methphase` end to end on the CPU oracle -- TEST INFRASTRUCTURE.

The same chain as the product's pipeline, with every compute step taken from
the oracle: gaps (oracle.vcf_gaps, blockjoin.c:4442-4523), the -u pre-pass
(oracle.haptag_reads over each contig's reads, 1841-1898, qname first-wins
1880-1889, merged over contigs first-wins), per window the loader + worker
(oracle.load_reads + oracle.methphase: 1043-1173, 4217-4335), the joined
windows' qname -> hp table (first wins in (contig, window) order,
4408-4423 / 4572-4590), the dropped-interval rescue (tests/test_bam.py's
restatement of 2618-2694) and the epilogue (oracle/epilogue.py: lift,
blocks, GTF/TSV/VCF, 2250-2988).  Records come from the product's BAM
reader, which tests/test_bam.py checks against the test-side writer."""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def _text_lines(path):
    """the complete lines of a plain or gzipped text file (a last line without
    '\n' is never read, as the reference's buffered reader)"""
    import gzip
    raw = open(path, "rb").read()
    if raw[:2] == b"\x1f\x8b":
        raw = gzip.decompress(raw)
    return raw.decode().split("\n")[:-1]


def known_positions_multi(vcf_path, names):
    """The known positions recover_variant_phase_in_dropped_intervals scans per
    contig of the phase-block file (blockjoin.c:2618-2663): the var_storage
    branch of load_intervals_from_file (2150-2163) puts a line into the table
    of the contig its CHROM names, or -- a CHROM not among `names` -- into the
    table of the last name it found (i_ref_cache is only updated on a hit)."""
    from test_bam import _py_known
    out = {n: [] for n in names}
    cache = None
    for s in _text_lines(vcf_path):
        if not s or s.startswith("#"):
            continue
        tok = [t for t in s.split("\t") if t]
        if not tok:
            continue
        if tok[0] in out:
            cache = tok[0]
        if cache is not None:
            out[cache] += [k[0] for k in _py_known([s], tok[0])]
    return out


def input_haptag_text(bam_path, raw_hp):
    """-U's {prefix}.mp.input_haptag.tsv (blockjoin.c:4494-4517): every record
    in file order, its HP tag (get_hp_from_aln) + 1 and its -u tag + 1 (255
    when the qname is not in the table)."""
    from test_bamw import hp_tag_raw, parse_bam, qname
    _, bodies, _, _ = parse_bam(bam_path)
    rows = [f"{qname(b)}\t{hp_tag_raw(b) + 1}\t{raw_hp.get(qname(b), 254) + 1}\n" for b in bodies]
    return "#qname\treal_hp\ttagged_hp\n" + "".join(rows)


def methphase_files_oracle(bam_path, vcf_path, cfg, lcfg=None, untagged=False, recs_by_contig=None,
                           n_threads=8, intervals=None):
    """-> dict(decision, qname_hp, raw_hp, gtf, tsv, vcf, counts, input_haptag).
    recs_by_contig ({contig: [Rec]} as written) feeds the rescue restatement.
    cfg None: no -c, every contig's parameters from its coverage estimate.
    intervals=(path, fmt): --gtf / --tsv phase blocks (oracle.interval_gaps);
    with -u the VCF's contigs are still the pre-pass's (4446, 4460-4465);
    vcf_path None: no VCF (4706)."""
    import oracle
    from oracle import epilogue as ep
    from pomfret_amd import Config, LoadConfig
    from pomfret_amd.bam import BamFile, vcf_known_vars
    from test_bam import _py_rescue

    lcfg = lcfg or LoadConfig()
    contigs = oracle.interval_gaps(*intervals) if intervals else oracle.vcf_gaps(vcf_path)
    ucontigs = oracle.vcf_gaps(vcf_path) if untagged else []
    decision, qname_hp, raw_hp = [], {}, {}
    with BamFile(bam_path) as bam:
        covs = bam.estimate_coverage() if cfg is None else None

        def contig_cfg(name):
            # no -c: the contig's own estimate, looked up by name (4358-4390)
            if cfg is not None:
                return cfg
            return Config.from_coverage(int(covs[bam.tid(name)]), given=False)

        if untagged:
            for c in ucontigs:
                if bam.tid(c["name"]) < 0:
                    continue
                kv = vcf_known_vars(vcf_path, c["name"])
                if len(kv.pos) == 0:
                    continue
                reads, qn, _ = bam.fetch_contig_reads(c["name"])
                if not qn:
                    continue
                hp = oracle.haptag_reads(kv, reads)
                tab = {}
                for q, h in zip(qn, hp.tolist()):
                    tab.setdefault(q, int(h))
                for q, h in tab.items():
                    raw_hp.setdefault(q, h)
        for c in contigs:
            g = c["gaps"]
            if not g:
                continue
            if bam.tid(c["name"]) < 0:
                decision += [-1] * len(g)
                continue
            ws = np.array([a for a, _ in g], np.uint32)
            we = np.array([b for _, b in g], np.uint32)
            aln, qn, _ = bam.fetch_windows(c["name"], ws, we)
            if untagged:
                aln.hp = np.array([raw_hp.get(q, 254) for q in qn], np.uint8)
            wb, rec_read = oracle.load_reads(lcfg, aln)
            res = oracle.methphase(contig_cfg(c["name"]), wb, n_threads=n_threads)
            recs_of_read = np.flatnonzero(rec_read != 0xFFFFFFFF)
            dec = res.decision.astype(np.int8)
            decision += dec.tolist()
            ro = wb.win_read_off.astype(np.int64)
            for w in range(len(g)):
                if dec[w] < 0:
                    continue
                for i in range(ro[w], ro[w + 1]):
                    qname_hp.setdefault(qn[int(recs_of_read[i])], int(res.read_hp[i]))
    blocks = ep.phase_blocks(contigs, decision)
    vcf, counts = None, None
    if vcf_path:
        known = known_positions_multi(vcf_path, [c["name"] for c in contigs])
        rescue = []
        for c in contigs:
            if not c["dropped"] or recs_by_contig is None or c["name"] not in recs_by_contig:
                rescue.append({})
                continue
            rescue.append(_py_rescue(recs_by_contig[c["name"]], known[c["name"]], c["dropped"], qname_hp,
                                     raw_hp if untagged else None))
        vcf, counts = ep.vcf_bytes(vcf_path, contigs, blocks, rescue)
    return dict(decision=np.asarray(decision, np.int8), qname_hp=qname_hp, raw_hp=raw_hp,
                gtf=ep.gtf_text(contigs, blocks), tsv=ep.tsv_text(contigs, blocks), vcf=vcf, counts=counts,
                input_haptag=input_haptag_text(bam_path, raw_hp) if untagged else None)


def oracle_job_runner(bam_path, vcf_path, lcfg=None, n_threads=4, fetch_threads=1, inflate_threads=1):
    """runner(plan, kind, j) for pomfret_amd.pipeline.methphase_files_dist /
    the Plan steps: a job's result computed by the oracle instead of the
    device (CPU tests of the product's plan / shard / merge / write).
    fetch_threads: host reader threads per window job; inflate_threads: BGZF
    inflate threads of a -u job's whole-contig read (bgzf_mt)."""
    import oracle
    from pomfret_amd import LoadConfig
    from pomfret_amd.bam import BamFile, vcf_known_vars
    from pomfret_amd.pipeline import JOB_HAPTAG

    lcfg = lcfg or LoadConfig()

    def pack(names):
        enc = [q.encode() for q in names]
        off = np.zeros(len(enc) + 1, np.uint64)
        if enc:
            off[1:] = np.cumsum([len(q) for q in enc])
        return off, np.frombuffer(b"".join(enc), np.uint8).copy()

    def run(plan, kind, j):
        info = plan.job_info(kind, j)
        with BamFile(bam_path, threads=inflate_threads if kind == JOB_HAPTAG else 1) as bam:
            if kind == JOB_HAPTAG:
                kv = vcf_known_vars(vcf_path, info["contig_name"])
                tab = {}
                if len(kv.pos):
                    reads, qn, _ = bam.fetch_contig_reads(info["contig_name"])
                    if qn:
                        for q, h in zip(qn, oracle.haptag_reads(kv, reads).tolist()):
                            tab.setdefault(q, int(h))
                off, names = pack(list(tab))
                return dict(decision=np.zeros(0, np.int8), tag_off=np.zeros(1, np.uint64), off=off, names=names,
                            hp=np.array(list(tab.values()), np.uint8))
            ws, we, _ = plan.windows()
            w0, w1 = info["w0"], info["w1"]
            n = w1 - w0
            if bam.tid(info["contig_name"]) < 0:
                return dict(decision=np.full(n, -1, np.int8), tag_off=np.zeros(n + 1, np.uint64),
                            off=np.zeros(1, np.uint64), names=np.zeros(0, np.uint8), hp=np.zeros(0, np.uint8))
            aln, qn, _ = bam.fetch_windows(info["contig_name"], ws[w0:w1], we[w0:w1], threads=fetch_threads)
        if plan.opts.untagged:
            raw = plan.raw_hp()
            aln.hp = np.array([raw.get(q, 254) for q in qn], np.uint8)
        wb, rec_read = oracle.load_reads(lcfg, aln)
        res = oracle.methphase(info["cfg"], wb, n_threads=n_threads)
        recs = np.flatnonzero(rec_read != 0xFFFFFFFF)
        ro = wb.win_read_off.astype(np.int64)
        names, hp, cnt = [], [], []
        for w in range(n):
            k = 0
            if res.decision[w] >= 0:
                for i in range(ro[w], ro[w + 1]):
                    names.append(qn[int(recs[i])])
                    hp.append(int(res.read_hp[i]))
                    k += 1
            cnt.append(k)
        off, nb = pack(names)
        return dict(decision=res.decision.astype(np.int8), tag_off=np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint64),
                    off=off, names=nb, hp=np.array(hp, np.uint8))
    return run


def methphase_files_port(bam_path, vcf_path, out_prefix, cfg, lcfg=None, untagged=False, threads=16,
                         tsv=False, job_windows=0, intervals=None, write_input_tagging=False):
    """The CPU port of the whole `pomfret methphase` driver -- the bench's CPU
    side of the file-to-output legs, and a CPU check of the product's
    planner / merge / writers.  The product's C plan and writers run with
    --host-fetch semantics and `threads` as the reference's -t N: the host
    coverage pass of estimate_read_coverage_dirtyfast when cfg is None
    (blockjoin.c:951-1040) reads the BAM with `threads` BGZF inflate threads
    (bgzf_mt, 576-578; pf_bam_set_threads); every job is computed by the
    oracle: the -u pre-pass one contig per thread, each contig's read with
    threads / contigs inflate threads (the reference runs the contigs
    serially with -t N inflate threads, 2069-2080, 1848), then the window
    jobs in order, each fetched with `threads` reader threads and run on
    `threads` oracle threads over windows (the reference's kt_for runs
    contigs, 4560).  Writes the same outputs as methphase_files.  ->
    (result dict, seconds per phase)."""
    import time
    from concurrent.futures import ThreadPoolExecutor
    from pomfret_amd.pipeline import JOB_HAPTAG, JOB_WINDOWS, MODE_METHPHASE, Plan, _result, make_opts

    t0 = time.perf_counter()
    o = make_opts(bam_path, vcf_path, out_prefix, cfg, lcfg, untagged=untagged, tsv=tsv, threads=threads,
                  job_windows=job_windows, host_fetch=True, intervals=intervals,
                  write_input_tagging=write_input_tagging)
    plan = Plan(o)
    t1 = time.perf_counter()
    nj = plan.n_jobs(JOB_HAPTAG) if untagged else 0
    run = oracle_job_runner(bam_path, vcf_path, lcfg, n_threads=threads, fetch_threads=threads,
                            inflate_threads=max(1, threads // max(1, min(threads, nj))))
    try:
        if untagged:
            with ThreadPoolExecutor(max(1, min(threads, nj))) as ex:
                res = list(ex.map(lambda j: run(plan, JOB_HAPTAG, j), range(nj)))
            for j, r in enumerate(res):
                plan.set_result(JOB_HAPTAG, j, r)
            plan.merge_raw()
        t2 = time.perf_counter()
        for j in range(plan.n_jobs(JOB_WINDOWS)):
            plan.set_result(JOB_WINDOWS, j, run(plan, JOB_WINDOWS, j))
        t3 = time.perf_counter()
        plan.finish()
        out = _result(plan, MODE_METHPHASE)
        t4 = time.perf_counter()
    finally:
        plan.close()
    return out, dict(plan_s=t1 - t0, haptag_s=t2 - t1, windows_s=t3 - t2, finish_s=t4 - t3, total_s=t4 - t0)


def report_oracle(bam_path, vcf_path, cov, chunk_size, chunk_stride, lcfg=None, k=3, k_span=5000):
    """main_methreport (blockjoin.c:4901-5089) on the oracle: chunk windows
    of the raw gaps (restated loop, tests/test_windows.py), the per-contig
    parameters cov/10+1, 2x, cov/4+1, one decision per window -> the
    report.tsv text."""
    import oracle
    from pomfret_amd import Config, LoadConfig
    from pomfret_amd.bam import BamFile
    from test_windows import _report_windows_ref
    lcfg = lcfg or LoadConfig()
    rows = []
    with BamFile(bam_path) as bam:
        covs = bam.estimate_coverage() if cov <= 0 else None
        for ci, c in enumerate(oracle.vcf_gaps(vcf_path)):
            wins = _report_windows_ref(c["abs_start"], c["raw"], chunk_size, chunk_stride)
            if not wins:
                continue
            cv = cov if cov > 0 else (covs[ci] if ci < len(covs) else 0)
            sel = cv // 10 + 1
            cfg = Config(k=k, k_span=k_span, cov_for_selection=sel, cov_for_runtime=2 * sel, n_cand=cv // 4 + 1)
            if bam.tid(c["name"]) < 0:
                dec = [-1] * len(wins)
            else:
                aln, _, _ = bam.fetch_windows(c["name"], [a for a, _ in wins], [b for _, b in wins])
                wb, _ = oracle.load_reads(lcfg, aln)
                dec = oracle.methphase(cfg, wb, n_threads=4).decision.tolist()
            for (a, b), d in zip(wins, dec):
                rows.append(f"{c['name']}\t{a}\t{b}\t" + ("correct" if d == 0 else "switch" if d == 1 else "fail") + "\n")
    return "".join(rows)

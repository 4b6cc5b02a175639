set -o pipefail
mkdir -p gpurun_out/pc
PF_SYNTH_WORKERS=16 timeout -k 10 300 python3 tools/run_aln_once.py 1024 0 /tmp/pc_aln.npz 60 > gpurun_out/pc/gen.log 2>&1 || exit 10
export PF_BENCH_ALN_CACHE=/tmp/pc_aln.npz
for L in cur p0 cur p0; do
  if [ $L = p0 ]; then cp pomfret_amd/libpomfret_amd.so /tmp/cur.so 2>/dev/null; cp pomfret_amd/libpomfret_amd_p0.so pomfret_amd/libpomfret_amd.so; fi
  timeout -k 10 400 python3 -u bench.py --no-cpu --e2e-windows 0 --e2e-u-scale 0 --steps 10 --warmup 3 > gpurun_out/pc/$L.json 2> gpurun_out/pc/$L.err || exit 11
  python3 -c "import json; d=json.loads(open('gpurun_out/pc/$L.json').read().strip().splitlines()[-1]); print('$L', d['ms_per_step'], d['single_batch']['kernels_ms'] if 'kernels_ms' in d['single_batch'] else '', {k:v['ms_per_step'] for k,v in d['strong_projection'].items()})" | tee -a gpurun_out/pc/summary.txt
  if [ $L = p0 ]; then cp /tmp/cur.so pomfret_amd/libpomfret_amd.so; fi
done

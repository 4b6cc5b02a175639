# Round-1 measurement set on the GPU box (record-level bench = BASELINE configs[1]):
#   MEAS_TAG=m7 bash tools/measure_r01.sh
# bench with the CPU baseline; kernel-trace stats of the bench; FETCH_SIZE and
# WRITE_SIZE in separate passes over one record-level batch (generated and
# cached before any profiler starts); the HBM calibration kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${MEAS_TAG:-m7}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || exit 11
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python3 $R/bench.py --no-cpu --steps 20 > $O/bench_prof.json 2> $O/bench_prof.err || exit 12
PF_SYNTH_WORKERS=16 timeout -k 10 200 python3 $R/tools/run_aln_once.py 256 0 /tmp/aln256.npz > $O/gen.log 2>&1 || exit 13
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 $R/tools/run_aln_once.py 256 3 /tmp/aln256.npz > $O/fetch.log 2>&1 || exit 14
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 $R/tools/run_aln_once.py 256 3 /tmp/aln256.npz > $O/write.log 2>&1 || exit 15
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/calf -o calf --output-format csv -- $R/tools/ubench/hbm_cal > $O/calf.log 2>&1 || exit 16
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/calw -o calw --output-format csv -- $R/tools/ubench/hbm_cal > $O/calw.log 2>&1 || exit 17
echo done

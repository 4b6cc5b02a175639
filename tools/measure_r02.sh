# Round-2 measurement set (second pass, m2: device fetch in the tree) on the GPU box (the bench's N=1 workload: 1024
# windows at 60x, record level):
#   MEAS_TAG=m1 bash tools/measure_r02.sh
# bench (CPU baseline, legs); kernel-trace stats of the bench; FETCH_SIZE and
# WRITE_SIZE in separate passes over the same batch (generated and cached
# before any profiler starts); the HBM calibration kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${MEAS_TAG:-m2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || exit 11
echo bench done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python3 $R/bench.py --no-cpu --no-legs --steps 50 > $O/bench_prof.json 2> $O/bench_prof.err || exit 12
echo trace done
PF_SYNTH_WORKERS=16 timeout -k 10 300 python3 $R/tools/run_aln_once.py 1024 0 /tmp/aln1024.npz 60 > $O/gen.log 2>&1 || exit 13
echo gen done
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 $R/tools/run_aln_once.py 1024 3 /tmp/aln1024.npz 60 > $O/fetch.log 2>&1 || exit 14
echo fetch done
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 $R/tools/run_aln_once.py 1024 3 /tmp/aln1024.npz 60 > $O/write.log 2>&1 || exit 15
echo write done
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/calf -o calf --output-format csv -- $R/tools/ubench/hbm_cal > $O/calf.log 2>&1 || exit 16
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/calw -o calw --output-format csv -- $R/tools/ubench/hbm_cal > $O/calw.log 2>&1 || exit 17
rm -f /tmp/aln1024.npz

# end-to-end leg: kernel trace of the device fetch (BAM written first, outside the profiler)
timeout -k 10 300 python3 $R/tools/e2e_once.py 64 0 /tmp/pf_e2e.bam > $O/e2e_gen.log 2>&1 || exit 18
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/e2e -o e2e --output-format csv -- python3 $R/tools/e2e_once.py 64 3 /tmp/pf_e2e.bam > $O/e2e.log 2>&1 || exit 19
rm -f /tmp/pf_e2e.bam /tmp/pf_e2e.bam.bai
echo e2e done

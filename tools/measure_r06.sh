# Round-6 measurement set on the GPU box (the bench's N=1 headline workload,
# WORKLOADS["mix"] at 1024 windows, record level), run after bench.py:
#   bash tools/measure_r06.sh <tag>
# The batch is generated once, before any profiler starts (no forked
# generator workers under rocprofv3: VERDICT r05 hygiene), then: kernel-trace
# stats of the bench's step over that batch; FETCH_SIZE and WRITE_SIZE in
# separate passes with the HBM calibration kernel; SQ counter passes
# (instructions, waits) over a 256-window batch of the same workload.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-m14}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PF_SYNTH_WORKERS=16 timeout -k 10 300 python3 $R/tools/run_aln_once.py 1024 0 /tmp/aln1024.npz 60 > $O/gen.log 2>&1 || exit 13
PF_SYNTH_WORKERS=16 timeout -k 10 200 python3 $R/tools/run_aln_once.py 256 0 /tmp/aln256.npz 60 > $O/gen256.log 2>&1 || exit 18
echo gen done
PF_BENCH_ALN_CACHE=/tmp/aln1024.npz timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python3 $R/bench.py --no-cpu --no-legs --tiles 1 --split 1 --steps 50 --e2e-windows 0 --e2e-u-scale 0 > $O/bench_prof.json 2> $O/bench_prof.err || exit 12
echo trace done
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 $R/tools/run_aln_once.py 1024 3 /tmp/aln1024.npz 60 > $O/fetch.log 2>&1 || exit 14
echo fetch done
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 $R/tools/run_aln_once.py 1024 3 /tmp/aln1024.npz 60 > $O/write.log 2>&1 || exit 15
echo write done
[ -x $R/tools/ubench/hbm_cal ] || hipcc --offload-arch=gfx950 -O2 -o $R/tools/ubench/hbm_cal $R/tools/ubench/hbm_cal.hip || exit 21
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/calf -o calf --output-format csv -- $R/tools/ubench/hbm_cal > $O/calf.log 2>&1 || exit 16
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/calw -o calw --output-format csv -- $R/tools/ubench/hbm_cal > $O/calw.log 2>&1 || exit 17
echo cal done
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d $O/sq1 -o sq1 --output-format csv -- python3 $R/tools/run_aln_once.py 256 2 /tmp/aln256.npz 60 > $O/sq1.log 2>&1 || exit 19
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVES -d $O/sq2 -o sq2 --output-format csv -- python3 $R/tools/run_aln_once.py 256 2 /tmp/aln256.npz 60 > $O/sq2.log 2>&1 || exit 20
echo sq done
rm -f /tmp/aln256.npz /tmp/aln1024.npz

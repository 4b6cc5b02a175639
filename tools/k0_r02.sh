# K0 diagnosis at 60x (round 2): per-phase cycles (diagnostic build), SQ
# instruction/wait counters and HBM traffic passes over a 256-window batch.
#   bash tools/k0_r02.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-k0r02}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/tools/k0_prof.py 128 60 > $O/phases.txt 2>&1 || exit 10
PF_SYNTH_WORKERS=16 timeout -k 10 200 python3 $R/tools/run_aln_once.py 256 0 /tmp/aln256_60.npz 60 > $O/gen.log 2>&1 || exit 11
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d $O/p1 -o p1 --output-format csv -- python3 $R/tools/run_aln_once.py 256 2 /tmp/aln256_60.npz 60 > $O/p1.log 2>&1 || exit 12
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 $R/tools/run_aln_once.py 256 2 /tmp/aln256_60.npz 60 > $O/fetch.log 2>&1 || exit 13
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 $R/tools/run_aln_once.py 256 2 /tmp/aln256_60.npz 60 > $O/write.log 2>&1 || exit 14
rm -f /tmp/aln256_60.npz
echo done

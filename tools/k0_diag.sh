set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/d1; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
PF_SYNTH_WORKERS=16 timeout -k 10 300 python3 $R/tools/run_aln_once.py 256 0 /tmp/a.npz 60 > $O/gen.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/f0 -o f0 --output-format csv -- python3 $R/tools/run_aln_once.py 256 3 /tmp/a.npz 60 > $O/f0.log 2>&1 || exit 14
PF_K0_DIAG=1 timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/f1 -o f1 --output-format csv -- python3 $R/tools/run_aln_once.py 256 3 /tmp/a.npz 60 > $O/f1.log 2>&1 || exit 15
echo ok

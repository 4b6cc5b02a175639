# K3 main-kernel LDS budget sweep (problems per CU) on the 50 kb batch and the
# gap mix:  bash tools/k3_lds_fixed_sweep.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-k3lds}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PF_SYNTH_WORKERS=16 timeout -k 10 300 python3 $R/tools/mix_stats.py /tmp/f1024.npz 1024 fixed50 > $O/gen.log 2>&1 || exit 10
for L in 32768 40960 45056 47104 49152; do
  PF_DEBUG_FALLBACK=1 PF_K3_LDS=$L PF_K3_LDS_FB=73728 PF_PROF=0 timeout -k 10 200 python3 $R/tools/mix_stats.py /tmp/f1024.npz 1024 fixed50 > $O/f_$L.log 2>&1 || exit 11
  echo "fixed50 lds=$L $(grep -m1 '^kernels' $O/f_$L.log) $(grep -m2 deferred $O/f_$L.log | tail -1)"
done
rm -f /tmp/f1024.npz

# inflate A/B on the box: BAM-like and Huffman-only blocks (inflate_ab_data.py)
# and a small synthetic genome BAM (tests/_genome.py), for each harness build
# given (tools/ubench/inflate_ab*: variant A = _inf_a.hip, B = pf_inflate.hip),
# then the inflate and fetch GPU tests.   bash tools/ubench/infl_ab_run.sh inflate_ab_w4 ...
set -o pipefail
O=gpurun_out/infl
mkdir -p $O
python3 tools/ubench/inflate_ab_data.py /tmp/infl_bam.bin && python3 tools/ubench/inflate_ab_data.py /tmp/infl_huff.bin huff || exit 3
python3 -c "
import sys; sys.path.insert(0, 'tests')
import _genome
s = _genome.GenomeSpec(); s.contigs = (('chr1', 4_000_000),)
g = _genome.write_genome('/tmp/infl_g', s, workers=16)
print(g['bam'], g['bam_bytes'])
" > $O/gen.log 2>&1 || exit 4
B=$(head -1 $O/gen.log | cut -d' ' -f1)
for h in "$@"; do
  timeout -k 10 60 ./tools/ubench/$h /tmp/infl_bam.bin 256 > $O/${h}_bam.txt 2>&1 || exit 5
  timeout -k 10 60 ./tools/ubench/$h /tmp/infl_huff.bin 256 > $O/${h}_huff.txt 2>&1 || exit 6
  timeout -k 10 60 ./tools/ubench/$h $B 4 > $O/${h}_genome.txt 2>&1 || exit 7
done
timeout -k 10 300 python -u -m pytest tests/test_inflate_gpu.py tests/test_fetch_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log

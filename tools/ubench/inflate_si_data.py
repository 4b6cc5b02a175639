"""Test data for inflate_si: a BAM of the bench's genome model (tests/_genome:
60x, 30 kb reads with MM/ML, MD and QUAL strings, zlib level 6) over one
contig of argv[2] bases (default 3 Mb), written to argv[1] (+ .bai/.vcf)."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))
import _genome  # noqa: E402

L = int(sys.argv[2]) if len(sys.argv) > 2 else 3_000_000
spec = _genome.GenomeSpec(contigs=(("chr1", L),))
g = _genome.write_genome(sys.argv[1][:-4] if sys.argv[1].endswith(".bam") else sys.argv[1], spec, workers=16)
print(g["n_records"], g["bam_bytes"])

"""tools/ab_env.py against another build of the library: the same mix batch
and critical window, with pomfret_amd loading LIB (a .so in pomfret_amd/).

usage: python tools/ab_lib.py libpomfret_amd_variant.so 'NAME:VAR=val' ..."""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pomfret_amd._lib as L  # noqa: E402

L.LIB_PATH = os.path.join(os.path.dirname(L.LIB_PATH), sys.argv[1])
sys.argv = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "ab_env.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")

"""Build library variants for on-box A/B runs: one .so per -D set, into ablib/
(not the product library; MCDC_LIBRARY selects one; MCDC_AB_DIR=abship puts
them where gpurun sends them).
usage: python tools/build_variants.py name:DEF=1,DEF2=0 ..."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mapache_amd import build as B  # noqa: E402


def one(spec):
    name, _, defs = spec.partition(":")
    out = os.path.join(B.ROOT, OUTDIR, name + ".so")
    # (the product's build: the device-code guard and the library descriptors'
    # padding apply to variants too -- a plain hipcc build left a rocPRIM
    # kernel at an exact VGPR fill)
    return B.build_lib(force=True, defines=[d for d in defs.split(",") if d], out=out)


OUTDIR = os.environ.get("MCDC_AB_DIR", "ablib")  # (abship/: variants sent to the GPU box)

if __name__ == "__main__":
    os.makedirs(os.path.join(B.ROOT, OUTDIR), exist_ok=True)
    with ThreadPoolExecutor(4) as ex:
        for o in ex.map(one, sys.argv[1:]):
            print(o)

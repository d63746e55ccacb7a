"""Build an A/B variant of the step library with its own specialisation table.

usage: python tools/build_variant.py NAME [-DFLAG=V ...]
       MJH_STEP_SRC=<saved mjh_step.hip> python tools/build_variant.py NAME   (another revision)
  -> asimov-mjlab_amd/mjlab_amd/variants/libmjh_NAME.so (time it on the GPU box
     with MJH_LIB=<that path> python tools/kernel_bench.py ...)
The launch plan depends on the compile flags (MJH_PRESET, MJH_WPB, ...), so the
variant's model-specialised instances need a table generated from the
variant's own generic build: generic build (empty table) -> gen_spec.py with
that library -> final build.
"""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "asimov-mjlab_amd" / "csrc"
OUTD = ROOT / "asimov-mjlab_amd" / "mjlab_amd" / "variants"
name, flags = sys.argv[1], sys.argv[2:]
OUTD.mkdir(parents=True, exist_ok=True)
tmp = Path("/tmp/mjh_variants") / name
tmp.mkdir(parents=True, exist_ok=True)
srcs = [CSRC / f for f in ("mjh_step.hip", "mjh_envops.hip", "mjh_mdp.hip", "mjh_mgr.hip", "mjh_fuse.hip")]
if os.environ.get("MJH_STEP_SRC"):  # A/B against another revision of the step kernel (e.g. a saved HEAD copy)
  srcs[0] = Path(os.environ["MJH_STEP_SRC"])


def hipcc(table: Path, out: Path) -> None:
  cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", f"-I{ROOT / 'include'}", f"-I{CSRC}",
         f'-DMJH_SPEC_TABLE="{table}"', *flags, "-o", str(out), *map(str, srcs)]
  subprocess.run(cmd, check=True)


empty = tmp / "empty_table.h"
subprocess.run([sys.executable, str(ROOT / "tools" / "gen_spec.py"), "--empty", "--out", str(empty)], check=True)
gen = tmp / "libmjh_generic.so"
hipcc(empty, gen)
table = tmp / "spec_table.h"
subprocess.run([sys.executable, str(ROOT / "tools" / "gen_spec.py"), "--out", str(table)], check=True,
               env=dict(os.environ, MJH_LIB=str(gen)))
final = OUTD / f"libmjh_{name}.so"
hipcc(table, final)
print("built", final)

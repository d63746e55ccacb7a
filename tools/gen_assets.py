"""Regenerate the robot spec assets (resolved-spec JSON) from the reference MJCF.

The HIP path cannot read /root/reference on the GPU box, so the robot
descriptions mjlab ships (G1: src/mjlab/asset_zoo/robots/unitree_g1/xmls/g1.xml,
Go1: src/mjlab/asset_zoo/robots/unitree_go1/xmls/go1.xml) are parsed once here
by mjlab_amd's own MJCF reader and stored as resolved-spec JSON (defaults and
childclass already applied, fromto kept). Run from the repo root:

  python tools/gen_assets.py
"""

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))

from mjlab_amd.spec.mjcf import read_mjcf  # noqa: E402

REF = Path("/root/reference/src/mjlab/asset_zoo/robots")
OUT = ROOT / "asimov-mjlab_amd" / "mjlab_amd" / "assets"

SOURCES = {
  "unitree_g1.json": REF / "unitree_g1" / "xmls" / "g1.xml",
  "unitree_go1.json": REF / "unitree_go1" / "xmls" / "go1.xml",
}

if __name__ == "__main__":
  OUT.mkdir(parents=True, exist_ok=True)
  for name, src in SOURCES.items():
    spec = read_mjcf(src)
    (OUT / name).write_text(spec.to_json())
    print(f"wrote {OUT / name}: {len(spec.bodies)} bodies, {len(spec.geoms)} geoms")

"""Generate asimov-mjlab_amd/csrc/mjh_spec_table.h: model-specialised step
kernel constants for the benchmark models (run in the build container).

For each benchmark task the scene is compiled exactly as the env compiles it
(Scene(cfg.scene).compile() with the task's SimulationCfg applied), and the
generic library's launch plan (mjh_plan_ints: NVP, model sizes, per-world
layout, model-image offsets) is emitted as compile-time constants. At run time
a specialised instance is used only when a model's plan matches one of these
exactly, so a stale table can cost speed, never correctness.
usage: python tools/gen_spec.py   (needs the generic libmjh.so built first)
"""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
OUT = ROOT / "asimov-mjlab_amd" / "csrc" / "mjh_spec_table.h"
if "--out" in sys.argv:  # variant builds (tools/build_variant.py) write their own table
  OUT = Path(sys.argv[sys.argv.index("--out") + 1])
from mjlab_amd.sim.spec_table import EMPTY, layout_ints, plan_of, render  # noqa: E402

if "--empty" in sys.argv:  # before anything loads the (possibly stale) library
  OUT.write_text(EMPTY)
  sys.exit(0)

from mjlab_amd.scene.scene import Scene  # noqa: E402
from mjlab_amd.sim import Simulation, native  # noqa: E402
from mjlab_amd.tasks import load_env_cfg  # noqa: E402

TASKS = ("Mjlab-Velocity-Flat-Unitree-G1", "Mjlab-Velocity-Flat-Unitree-Go1", "Mjlab-Tracking-Flat-Unitree-G1")


def task_plan(task: str) -> list[int]:
  cfg = load_env_cfg(task)
  cfg.scene.num_envs = 1
  cfg.sim.specialize = "off"  # the plan only: no plugin lookup
  sim = Simulation(1, cfg.sim, Scene(cfg.scene, device="cpu").compile(), "cpu")
  return plan_of(native.lib(), ctypes.addressof(sim._mstruct))


def main() -> None:
  plans, names = [], []
  for t in TASKS:
    p = task_plan(t)
    if p not in plans:
      plans.append(p)
      names.append(t)
  OUT.write_text(render(plans, names, layout_ints(native.lib())))
  print(f"wrote {OUT.name}: {len(plans)} specialisations ({', '.join(names)})")


if __name__ == "__main__":
  main()

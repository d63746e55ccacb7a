"""Build the launch plugin (model-specialised step kernel, mjlab_amd/sim/jit.py) for a
task's model ahead of time, so a GPU run finds it in the cache instead of compiling.

usage: python tools/jit_build.py [TASK] [--framepos BODY]...
  --framepos BODY adds a BuiltinSensorCfg framepos on the robot's BODY (the model the
  GPU test tests/test_gpu_jit.py runs: the G1 velocity task plus one pelvis framepos,
  a sensor outside the built-in specialisations' set). Runs on the CPU container.
"""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
from mjlab_amd.scene.scene import Scene  # noqa: E402
from mjlab_amd.sensor.builtin_sensor import BuiltinSensorCfg, ObjRef  # noqa: E402
from mjlab_amd.sim import Simulation, jit, native  # noqa: E402
from mjlab_amd.sim.spec_table import plan_of  # noqa: E402
from mjlab_amd.tasks import load_env_cfg  # noqa: E402


def task_model(task: str, framepos=()):
  cfg = load_env_cfg(task)
  cfg.scene.num_envs = 1
  cfg.scene.sensors = tuple(cfg.scene.sensors) + tuple(
    BuiltinSensorCfg(name=f"{b}_pos", sensor_type="framepos", obj=ObjRef(type="xbody", name=b, entity="robot"))
    for b in framepos)
  return cfg, Scene(cfg.scene, device="cpu").compile()


def main() -> None:
  args = sys.argv[1:]
  task = args[0] if args and not args[0].startswith("--") else "Mjlab-Velocity-Flat-Unitree-G1"
  framepos = [args[i + 1] for i, a in enumerate(args) if a == "--framepos"]
  cfg, m = task_model(task, framepos)
  cfg.sim.specialize = "off"
  sim = Simulation(1, cfg.sim, m, "cpu")
  addr = ctypes.addressof(sim._mstruct)
  if native.lib().mjh_spec_index(addr) >= 0:
    print(f"{task}: a built-in specialisation covers this model; nothing to build")
    return
  path = jit.compile_plugin(plan_of(native.lib(), addr), name=task + "".join(f"+framepos:{b}" for b in framepos))
  print("plugin:", path)


if __name__ == "__main__":
  main()

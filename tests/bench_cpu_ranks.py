"""bench.py's multi-rank path on CPU (TEST INFRASTRUCTURE ONLY).

`python tests/bench_cpu_ranks.py --gpus 2 --device cpu ...` runs bench.main with
the float64 oracle attached as each rank's physics (tests/oracle_sim.py): the
same spawn (bench.spawn_ranks re-launches this script under
torch.distributed.run), WORLD_SIZE check, barriers, MAX all-reduce of the
timed window, per-step packed all-gather and rank-0 JSON line as on the GPU
box, over gloo instead of RCCL. Never used by the product path."""

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from tests import oracle_sim  # noqa: E402


def hook(env) -> None:
  oracle_sim.attach(env.sim, env.event_manager.domain_randomization_fields)


if __name__ == "__main__":
  bench.main(env_hook=hook)

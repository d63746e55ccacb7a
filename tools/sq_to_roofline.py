"""profiles/step_kernel_sq.json for bench.py's roofline_valu block, from a
tools/pmc_summary.py output: SQ_INSTS_VALU summed over the step-kernel
instances of one physics step (the fused kernel, or the split step's position
and velocity kernels), per launch.

usage: python tools/sq_to_roofline.py <sq_summary.json> <task> <num_envs> <source-tag> [out]"""
import json
import sys
from pathlib import Path

src, task, n, tag = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
out = Path(sys.argv[5]) if len(sys.argv) > 5 else Path(__file__).resolve().parents[1] / "profiles" / "step_kernel_sq.json"
s = json.load(open(src))
pk = {k: v for k, v in s.get("per_kernel", {}).items() if "step_kernel" in k}
ins = sum(v.get("SQ_INSTS_VALU", 0.0) for v in pk.values())
# latency share: wave-cycles spent waiting (any dependency) over all wave-cycles
wait = sum(v.get("SQ_WAIT_ANY", 0.0) for v in pk.values()) or s.get("SQ_WAIT_ANY", 0.0)
cyc = sum(v.get("SQ_WAVE_CYCLES", 0.0) for v in pk.values()) or s.get("SQ_WAVE_CYCLES", 0.0)
out.write_text(json.dumps({"task": task, "num_envs": n, "valu_insts_per_launch": ins, "kernels": sorted(pk),
                           "wait_any_frac": (wait / cyc) if cyc else None, "sq_wait_any": wait, "sq_wave_cycles": cyc,
                           "source": tag}, indent=1) + "\n")
print("wrote", out, ins)

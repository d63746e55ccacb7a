"""Average per-dispatch PMC counters of one kernel from rocprofv3 counter_collection CSVs.

usage: python tools/pmc_summary.py <kernel-substring> <skip> file1.csv [file2.csv ...]
Prints one JSON object {counter: mean value per dispatch} over the matching
dispatches after the first <skip> (settling launches), plus derived ratios
per wave when SQ_WAVES is present (SQ_*_CYCLES count quad-cycles on gfx950,
MI355X_MICROARCH.md "s_memtime tick vs SQ PMC units").
"""
import csv
import json
import sys


def main() -> None:
  pat, skip, files = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
  acc: dict[str, dict[int, float]] = {}
  per_kernel: dict[str, dict[str, dict[int, float]]] = {}
  for f in files:
    for r in csv.DictReader(open(f)):
      if pat not in r["Kernel_Name"]:
        continue
      d = int(r["Dispatch_Id"])
      acc.setdefault(r["Counter_Name"], {})
      acc[r["Counter_Name"]][d] = acc[r["Counter_Name"]].get(d, 0.0) + float(r["Counter_Value"])
      pk = per_kernel.setdefault(r["Kernel_Name"], {}).setdefault(r["Counter_Name"], {})
      pk[d] = pk.get(d, 0.0) + float(r["Counter_Value"])
  out = {}
  for name, per in sorted(acc.items()):
    ks = sorted(per)[skip:] or sorted(per)
    out[name] = sum(per[k] for k in ks) / len(ks)
    out.setdefault("_dispatches", {})[name] = len(ks)
  w = out.get("SQ_WAVES")
  if w:
    der = {}
    for name in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                 "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                 "SQ_ACTIVE_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_MFMA", "SQ_INSTS_VALU_MFMA_F32"):
      if name in out:
        der[name + "_per_wave"] = out[name] / w
    out["derived"] = der
  # per kernel instance (a split step launches two step kernels per physics step)
  def mean_after_skip(per: dict[int, float]) -> float:
    ks = sorted(per)[skip:] or sorted(per)
    return sum(per[k] for k in ks) / len(ks)

  out["per_kernel"] = {k: {c: mean_after_skip(v) for c, v in cs.items()} for k, cs in per_kernel.items()}
  print(json.dumps(out, indent=1))


if __name__ == "__main__":
  main()

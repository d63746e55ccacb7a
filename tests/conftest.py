import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
# the test scenes' step kernels: a launch plugin only if one is already built
# (tests/test_gpu_jit.py asks for "auto" itself); no hipcc run inside a test
os.environ.setdefault("MJH_SPECIALIZE", "cached")
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
  config.addinivalue_line("markers", "gpu: needs an MI355X (HIP step library on cuda:0)")


@pytest.fixture(scope="session")
def gpu():
  import torch

  if not torch.cuda.is_available():
    pytest.skip("no GPU")
  return "cuda:0"


def pytest_collection_modifyitems(config, items):
  import torch

  if torch.cuda.is_available():
    return
  skip = pytest.mark.skip(reason="needs a GPU (run with -m gpu on the MI355X box)")
  for it in items:
    if "gpu" in it.keywords:
      it.add_marker(skip)


@pytest.fixture(autouse=True)
def _solver_decision_fraction():
  """Over all compare_step calls of one test: the worlds whose warm-start pick
  differs from the float64 oracle's own (outside float32 ties, within float32
  noise; beyond it compare_step fails the call) are at most DECISION_FRAC of
  the worlds checked, with two near-ties admitted per test (and at most
  DECISION_FRAC over the whole session: pytest_sessionfinish). Stop decisions
  within float32 noise are reported, not bounded (tests/scenes.py docstring)."""
  mod = sys.modules.get("tests.scenes")
  start = len(mod.PARITY_LOG) if mod is not None else 0
  yield
  mod = sys.modules.get("tests.scenes")
  if mod is None:
    return
  recs = mod.PARITY_LOG[start:]
  mis = sum(r["warm_mismatch"] for r in recs)
  tot = sum(r["warm_worlds"] for r in recs)
  if mis > max(2, int(mod.DECISION_FRAC * tot)):
    pytest.fail(f"solver warm-start pick differs from the float64 oracle's in {mis} of {tot} world-steps "
                f"(> {mod.DECISION_FRAC:.0%}; all within float32 noise of the comparison)")


def pytest_sessionfinish(session, exitstatus):
  """Session-wide: warm-start picks that differ from the float64 oracle's
  (outside float32 ties) are at most DECISION_FRAC of all world-steps checked."""
  mod = sys.modules.get("tests.scenes")
  if mod is None or not mod.PARITY_LOG:
    return
  mis = sum(r["warm_mismatch"] for r in mod.PARITY_LOG)
  tot = sum(r["warm_worlds"] for r in mod.PARITY_LOG)
  if tot and mis > mod.DECISION_FRAC * tot:
    print(f"\nsolver warm-start picks differ from the float64 oracle's in {mis} of {tot} world-steps (> 1%)")
    session.exitstatus = 1


def pytest_terminal_summary(terminalreporter, exitstatus, config):
  """One line per parity test (every tests/scenes.compare_step call it made):
  the worst per-world bound ratio (1.0 = at the bound), and the counts of
  worlds exempted from the hard bounds (unconverged at the cap / parallel
  line-search choices beyond the float32 noise), of integer mismatches, and
  of solver-decision mismatches against the float64 oracle's own decisions
  (explained by float32 noise / not)."""
  try:
    from tests.scenes import PARITY_LOG
  except Exception:
    return
  if not PARITY_LOG:
    return
  agg: dict[str, dict] = {}
  for r in PARITY_LOG:
    a = agg.setdefault(r["test"].split("::")[-1], dict(calls=0, worlds=0, worst=0.0, capped=0, ls=0, imis=0, stop=0, warm=0,
                                                        unexpl=0, dchk=0, nit=0, sw=0, ww=0, dworst=0.0, early=0, tie=0,
                                                        soft=0, cver=0, chard=0))
    a["calls"] += 1
    a["worlds"] += r["worlds"]
    a["worst"] = max(a["worst"], r["worst_bound"])
    a["soft"] += r.get("soft_over", 0)
    a["capped"] += r["capped"]
    a["cver"] += r.get("capped_verified", 0)
    a["chard"] += r.get("capped_held_hard", 0)
    a["ls"] += r["ls_outliers"]
    a["imis"] += r["int_mismatch"]
    a["stop"] += r["stop_mismatch"]
    a["warm"] += r["warm_mismatch"]
    a["unexpl"] += r["decision_unexplained"]
    a["dchk"] += r["decisions_checked"]
    a["nit"] += r["niter_differs"]
    a["sw"] += r["stop_worlds"]
    a["early"] += r["stop_early"]
    a["tie"] += r["warm_tie"]
    a["ww"] += r["warm_worlds"]
    a["dworst"] = max(a["dworst"], r["decision_worst"])
  tr = terminalreporter
  tr.write_sep("-", "parity exemptions (worlds; worst = max per-world error / hard bound; soft = admitted over the soft bound)")
  tot = dict(worlds=0, capped=0, ls=0, imis=0, stop=0, early=0, warm=0, tie=0, unexpl=0, sw=0, ww=0, worst=0.0, soft=0,
             cver=0, chard=0)
  for name, a in agg.items():
    tr.write_line(f"{name[:60]:60s} w={a['worlds']} worst={a['worst']:.2f} soft={a['soft']} capped={a['capped']} "
                  f"(re-run converged {a['cver']}) capped_held_hard={a['chard']} ls_out={a['ls']} "
                  f"int_mis={a['imis']} stop_noise={a['stop']}/{a['sw']} (early {a['early']}) warm_mis={a['warm']}/{a['ww']} "
                  f"warm_tie={a['tie']} "
                  f"dec_worst={a['dworst']:.2f} unexpl={a['unexpl']} niter_diff={a['nit']}")
    for k in tot:
      tot[k] = max(tot[k], a[k]) if k == "worst" else tot[k] + a[k]
  for r in getattr(sys.modules.get("tests.scenes"), "ITER_LOG", []):
    tr.write_line(f"ITERATIONS {r['test'].split('::')[-1][:60]:60s} device {r['device']:.3f} oracle_f32 "
                  f"{r['oracle_f32']:.3f} oracle_f64 {r['oracle_f64']:.3f} ok={r['ok']}")
  tr.write_line(f"PARITY TOTAL worlds={tot['worlds']} worst_bound={tot['worst']:.2f} soft_over={tot['soft']} capped={tot['capped']} "
                f"capped_rerun_converged={tot['cver']} capped_unverified={tot['capped'] - tot['cver']} "
                f"({(tot['capped'] - tot['cver']) / max(1, tot['worlds']):.2%}) capped_held_hard={tot['chard']} "
                f"ls_outliers={tot['ls']} int_mismatch={tot['imis']} stop_within_noise={tot['stop']}/{tot['sw']} "
                f"(early {tot['early']}) warm_mismatch={tot['warm']}/{tot['ww']} warm_ties={tot['tie']} "
                f"decision_unexplained={tot['unexpl']}")

"""Offline study of world-order cost predictors (input: tools/phase_profile.py
DUMP=... npz): workgroup-max mean of step t+1 cycles when worlds are ordered by
a predictor computed from step t."""
import sys

import numpy as np

z = np.load(sys.argv[1])
tot1, tot2, niter, nefc, ncon = z["tot1"].astype(float), z["tot2"].astype(float), z["niter"].astype(float), \
  z["nefc"].astype(float), z["ncon"].astype(float)
N = len(tot2)
M8 = (N // 8) * 8


def wgmax(key):
  o = np.argsort(-key, kind="stable")
  return tot2[o][:M8].reshape(-1, 8).max(1).mean()


X = np.stack([np.ones(N), niter, nefc, niter * nefc, ncon, nefc ** 2, niter ** 2], 1)
coef, *_ = np.linalg.lstsq(X, tot1, rcond=None)
print("mean", tot2.mean(), "identity", wgmax(-np.arange(N)), "true", wgmax(tot2))
for name, key in [("(niter+2)*nefc", (niter + 2) * nefc), ("prev cycles", tot1), ("fit(niter,nefc,...)", X @ coef),
                  ("nefc", nefc), ("niter", niter), ("(niter+1)*nefc", (niter + 1) * nefc), ("(niter+4)*nefc", (niter + 4) * nefc),
                  ("(niter+2)*(nefc+10)", (niter + 2) * (nefc + 10)), ("0.5 rank mix", np.argsort(np.argsort(tot1)) + np.argsort(np.argsort((niter + 2) * nefc)))]:
  print(f"{name:24s} {wgmax(key):10.0f}")

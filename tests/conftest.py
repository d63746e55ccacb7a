import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
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

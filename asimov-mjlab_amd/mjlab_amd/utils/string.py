"""Name/regex resolution helpers with mjlab's matching rules.

``resolve_expr``/``filter_exp``/``resolve_field``: first-match-wins prefix
regex matching (``re.match``), as in ``src/mjlab/utils/string.py:7-47``.
``resolve_matching_names``: full-match, one-to-one check, optional order
preservation, as in Isaac Lab's helper vendored at
``src/mjlab/third_party/isaaclab/isaaclab/utils/string.py:178-271``.
"""

from __future__ import annotations

import re
from typing import Any, Sequence


def resolve_expr(pattern_map: dict[str, Any], names: Sequence[str], default_val: Any = 0.0) -> tuple:
  patterns = [(re.compile(p), v) for p, v in pattern_map.items()]
  out = []
  for n in names:
    for pat, v in patterns:
      if pat.match(n):
        out.append(v)
        break
    else:
      out.append(default_val)
  return tuple(out)


def filter_exp(exprs: Sequence[str], names: Sequence[str]) -> tuple[str, ...]:
  pats = [re.compile(e) for e in exprs]
  return tuple(n for n in names if any(p.match(n) for p in pats))


def resolve_field(field: Any, names: Sequence[str], default_val: Any = 0) -> tuple:
  if isinstance(field, dict):
    return resolve_expr(field, names, default_val)
  return tuple([field] * len(names))


def resolve_matching_names(
  keys: str | Sequence[str], list_of_strings: Sequence[str], preserve_order: bool = False
) -> tuple[list[int], list[str]]:
  if isinstance(keys, str):
    keys = [keys]
  idx, names, key_idx = [], [], []
  matched_by: list[str | None] = [None] * len(list_of_strings)
  key_hits: list[list[str]] = [[] for _ in keys]
  for ti, s in enumerate(list_of_strings):
    for ki, k in enumerate(keys):
      if re.fullmatch(k, s):
        if matched_by[ti]:
          raise ValueError(f"Multiple matches for '{s}': '{matched_by[ti]}' and '{k}'!")
        matched_by[ti] = k
        idx.append(ti)
        names.append(s)
        key_idx.append(ki)
        key_hits[ki].append(s)
  if preserve_order:
    order = sorted(range(len(idx)), key=lambda i: (key_idx[i], i))
    idx = [idx[i] for i in order]
    names = [names[i] for i in order]
  unmatched = [k for k, hits in zip(keys, key_hits) if not hits]
  if unmatched:
    raise ValueError(
      f"Not all regular expressions are matched! Unmatched: {unmatched}. Available: {list(list_of_strings)}"
    )
  return idx, names


def resolve_matching_names_values(
  data: dict[str, Any], list_of_strings: Sequence[str], preserve_order: bool = False
) -> tuple[list[int], list[str], list[Any]]:
  if not isinstance(data, dict):
    raise TypeError(f"Input argument `data` should be a dictionary. Received: {data}")
  keys = list(data.keys())
  idx, names = resolve_matching_names(keys, list_of_strings, preserve_order)
  values = []
  for n in names:
    for k in keys:
      if re.fullmatch(k, n):
        values.append(data[k])
        break
  return idx, names, values

#!/bin/bash
# Build kernel variants for A/B timing: specs are PRESET_WPB[_FLAGS], where
# FLAGS letters: i = inline solver helpers, c = inline narrowphase.
set -e
cd "$(dirname "$0")/.."
out=asimov-mjlab_amd/mjlab_amd/variants
mkdir -p $out
for spec in "$@"; do
  IFS=_ read -r p w f <<< "$spec"
  extra=""
  [[ "$f" == *i* ]] && extra="$extra -DMJH_SOLVER_INLINE=__forceinline__"
  [[ "$f" == *c* ]] && extra="$extra -DMJH_COLL_INLINE=__forceinline__"
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude -DMJH_PRESET=$p -DMJH_WPB=$w $extra \
    -o $out/libmjh_$spec.so asimov-mjlab_amd/csrc/mjh_step.hip asimov-mjlab_amd/csrc/mjh_envops.hip asimov-mjlab_amd/csrc/mjh_mdp.hip asimov-mjlab_amd/csrc/mjh_mgr.hip &
done
wait

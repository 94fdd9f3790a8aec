#!/bin/bash
# Time the stationary kernel of several library builds in one GPU session (A/B experiments).
# usage: tools/ab_time.sh lib1.so lib2.so ...   (paths relative to llama-fft_amd/lib)
cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib (pass $rep)"
    BCFFT_LIB_PATH=llama-fft_amd/lib/$lib timeout -k 10 120 python3 -u tools/time_algos.py stationary 2>&1 | grep -v amdgpu.ids || exit 1
  done
done

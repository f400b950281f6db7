#!/bin/bash
# Build tools/kbench_attn.hip with compiler-flag variants and time the library attention kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for FL in "" ${KB_FLAGS:-}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics $FL tools/kbench_attn.hip -o /tmp/ka$i 2>/dev/null || { echo "build failed: $FL"; exit 1; }
  echo "== flags: [$FL]"
  KB_ONLY=lib timeout -k 10 120 /tmp/ka$i || exit 1
  i=$((i+1))
done

#!/bin/bash
# Host-side AddressSanitizer + UBSan build of libhgk (-Xarch_host: the sanitizers instrument the
# host code only; GPU sanitizers are not available on this pool), linked into
# scripts/asan_host_check.cpp and run. Without a GPU every kernel launch fails cleanly AFTER the
# host work that precedes it (validation, planning, descriptor packing), which is what is checked.
# Objects are cached (rebuilt when a source or header is newer). CPU-only; tests/test_host_sanitizer.py.
# usage: bash scripts/asan_host.sh [outdir]
set -eo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=${1:-$R/build/asan}
mkdir -p "$O"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN_HOST="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer"
FLAGS="-O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include $SAN_HOST"
HDRS="$R/include/hgk.h $R/progressive_process_for_human_pose_estimation_amd/csrc/hgk_common.h"
objs=()
pids=()
for src in "$R"/progressive_process_for_human_pose_estimation_amd/csrc/*.hip "$R"/progressive_process_for_human_pose_estimation_amd/csrc/*.cpp; do
  obj="$O/$(basename "$src").o"
  objs+=("$obj")
  stale=0
  [ -f "$obj" ] || stale=1
  for dep in "$src" $HDRS; do [ "$dep" -nt "$obj" ] && stale=1; done
  if [ $stale = 1 ]; then "$HIPCC" $FLAGS -c "$src" -o "$obj" & pids+=($!); fi
done
for p in "${pids[@]}"; do wait "$p"; done
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined"
/opt/rocm/lib/llvm/bin/clang++ -O1 -g -std=c++17 $SAN -I"$R/include" -c "$R/scripts/asan_host_check.cpp" -o "$O/check.o"
"$HIPCC" $SAN --offload-arch=gfx950 "$O/check.o" "${objs[@]}" -o "$O/asan_host_check"
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$O/asan_host_check"

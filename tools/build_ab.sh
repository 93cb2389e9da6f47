#!/bin/bash
# Build an alternative libaninerf_hip.so with extra -D flags into ab/NAME.so (same-box A/B through
# tools/gpu.sh ab:NAME): tools/build_ab.sh NAME "-DFOO=1 -DBAR=0"
set -e
NAME=$1
FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=/tmp/ab_$NAME
mkdir -p "$OUT" "$ROOT/ab"
SRCS=$(sed -n 's/^SRCS := //p; s/^        \(.*\)$/\1/p' "$ROOT/Makefile" | tr -d '\\' | tr ' ' '\n' | grep '\.hip$' | sed 's#\$(SRC_DIR)#animatable_nerf_amd/csrc#')
objs=()
pids=()
for s in $SRCS; do
  o=$OUT/$(basename "$s" .hip).o
  objs+=("$o")
  (cd "$ROOT" && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -Iinclude $FLAGS -c "$s" -o "$o") &
  pids+=($!)
  if [ ${#pids[@]} -ge 8 ]; then wait "${pids[0]}"; pids=("${pids[@]:1}"); fi
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/ab/$NAME.so" "${objs[@]}"
echo "built ab/$NAME.so"

#!/bin/bash
# Build libcgs_kernels.so of a git revision (default HEAD) into scratch/ab/<rev>/ for in-process
# library A/Bs (tools/probes/lib_ab.py). CPU only (hipcc cross-compiles gfx950).
#   tools/build_rev_lib.sh [rev]
set -e
cd "$(dirname "$0")/.."
rev="${1:-HEAD}"
sha=$(git rev-parse --short "$rev")
out="scratch/ab/$sha"
mkdir -p "$out/src"
git archive "$rev" comfy_gen_server_amd/csrc/kernels | tar -x -C "$out/src"
k="$out/src/comfy_gen_server_amd/csrc/kernels"
objs=()
for s in "$k"/*.hip; do
  o="$out/$(basename "$s").o"
  objs+=("$o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -mcode-object-version=5 \
    -Wno-unused-result -munsafe-fp-atomics -c "$s" -o "$o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -o "$out/libcgs_kernels.so" "${objs[@]}"
rm -rf "$out/src" "$out"/*.o
echo "$out/libcgs_kernels.so"

#!/bin/bash
# Builds variant libraries next to libmmpt.so for A/B runs (MMPT_LIB=...; never used by the
# product path): lib/diag/libmmpt_<name>.so for each "<name>:<source>:<extra hipcc flags>"
# argument — <source> (gemm | attention | layernorm | misc) rebuilt with the flags, every
# other object as built by the Makefile.
set -euo pipefail
cd "$(dirname "$0")/../../multimodal_llm_pretraining_amd/csrc"
[ -n "${NOMAKE:-}" ] || make -s -j8 > /dev/null
mkdir -p ../lib/diag
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; src=${rest%%:*}; flags=${rest#*:}
  (
    objs=""
    for o in capi gemm layernorm attention misc quant batch; do
      if [ "$o" = "$src" ]; then objs="$objs ../lib/diag/${src}_$name.o"; else objs="$objs ../lib/obj/$o.o"; fi
    done
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include $flags \
        -c $src.hip -o ../lib/diag/${src}_$name.o &&
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs -o ../lib/diag/libmmpt_$name.so &&
    rm -f ../lib/diag/${src}_$name.o
  ) &
done
wait

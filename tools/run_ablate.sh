#!/bin/bash
# Layer timings of the product library and the ablation variants under tp-gan_amd/ablate/
# (make ablate ...): bash tools/run_ablate.sh <tag> <variant dirs...> -- <bench_layers args>
TAG=$1; shift
V=()
while [[ $# -gt 0 && $1 != -- ]]; do V+=("$1"); shift; done
shift
A="layers $*"
steps=("$A")
for v in "${V[@]}"; do steps+=("TPG_LIB_PATH=tp-gan_amd/ablate/$v/libtpgan_hip.so $A"); done
exec bash tools/gpu.sh "$TAG" "${steps[@]}"

#!/bin/bash
# Build diagnostic variants of libdclip.so into ab/ (gitignored; they travel to the GPU box):
#   bash tools/build_ab_variants.sh NAME "-DFLAG ..." [NAME2 "-D..."]
# Only attention.hip and attention_dkdv6.hip are rebuilt with the flags; the rest are the
# product objects from denseclip_vit_multimodal_amd/csrc/build.
set -e
cd "$(dirname "$0")/.."
C=denseclip_vit_multimodal_amd/csrc
make -C $C -j8 > /dev/null
mkdir -p ab
while [ $# -gt 0 ]; do
  name=$1; flags=$2; shift 2
  d=ab/$name; mkdir -p $d
  F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -fno-slp-vectorize -fno-honor-nans -mllvm -amdgpu-mfma-vgpr-form"
  /opt/rocm/bin/hipcc $F $flags -c $C/attention.hip -o $d/attention.o &
  /opt/rocm/bin/hipcc $F $flags -c $C/attention_dkdv6.hip -o $d/attention_dkdv6.o &
  wait
  objs=""
  for o in capi layernorm gemm attention_fp8 misc headloss data; do objs="$objs $C/build/$o.o"; done
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $d/attention.o $d/attention_dkdv6.o -o $d/libdclip.so
  echo "built $d/libdclip.so ($flags)"
done

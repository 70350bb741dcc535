#!/bin/bash
# Build a debug/instrumented variant of the HIP library next to the product one (host-side, here, not on the box):
#   tools/build_variant.sh NAME "-DFLAG ..."  ->  fmdiff/lib/variants/libfmdiff_NAME.so  (select with FMD_LIB=...)
set -e
cd "$(dirname "$0")/../flow-matching-and-diffusion-models_amd"
name=$1; shift
out=fmdiff/lib/variants; mkdir -p $out build/var_$name
objs=()
for f in csrc/*.hip; do
  o=build/var_$name/$(basename $f).o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-slp-vectorize -I csrc -I ../include $@ -c $f -o $o &
  objs+=($o)
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC ${objs[@]} -o $out/libfmdiff_$name.so
echo "built $out/libfmdiff_$name.so"

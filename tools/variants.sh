#!/bin/bash
# Build engine variants with different compile-time map tunables (CPU side):
#   tools/variants.sh NAME "-DWC_MAP_STICKY_CAP=0 -DWC_MAP_FILL_EIGHTHS=6" [NAME2 "FLAGS2" ...]
# -> cuda_mapreduce_amd/lib/variants/libwc_NAME.so; run with WC_LIB=<path> python bench.py
set -e
cd "$(dirname "$0")/.."
mkdir -p cuda_mapreduce_amd/lib/variants build/variants
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  d=build/variants/$name; mkdir -p $d
  objs=""
  for f in src/kernels/*.hip; do
    o=$d/$(basename $f .hip).o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Isrc $flags -c $f -o $o &
    objs="$objs $o"
  done
  cpp=""
  for f in src/common/*.cpp src/engine/*.cpp src/dist/*.cpp src/cpu/*.cpp src/io/*.cpp src/output/*.cpp src/capi.cpp; do
    o=$d/cpp_$(echo $f | tr '/' '_' | sed 's/\.cpp$//').o
    g++ -O3 -std=c++17 -fPIC -D__HIP_PLATFORM_AMD__ -Iinclude -Isrc -I/opt/rocm/include $flags -c $f -o $o &
    cpp="$cpp $o"
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o cuda_mapreduce_amd/lib/variants/libwc_$name.so $objs $cpp \
    -L/opt/rocm/lib -lrccl -lrocprofiler-sdk-roctx -lamdhip64 -lpthread -Wl,-rpath,/opt/rocm/lib
  echo built $name
done

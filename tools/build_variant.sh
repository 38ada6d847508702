#!/bin/bash
# A/B build: recompile one instantiation unit (default pbh_inst_a, d <= 4)
# with extra -D flags and link it with the other objects of the current
# build into probayes_amd/libpbhip_NAME.so (load it with PBHIP_LIB=...).
# usage: tools/build_variant.sh NAME "-DFLAG=v ..." [unit]
set -euo pipefail
name=$1; flags=$2; unit=${3:-pbh_inst_a}
cd "$(dirname "$0")/../probayes_amd/csrc"
B=build_$name
mkdir -p $B
CXXFLAGS="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -Wall -Wno-unused-function -I../../include"
HIPCC=/opt/rocm/bin/hipcc ARCH=gfx950 ./hip_e64.sh $unit.hip $B/$unit.o $CXXFLAGS $flags
objs=$(ls build/*.o | grep -v "/$unit.o" | grep -v "\.dev\.")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libpbhip_$name.so $B/$unit.o $objs -lrccl
echo "built libpbhip_$name.so ($unit $flags)"

#!/bin/bash
# build lib_<name>.so: flow.hip with extra flags, other objects from the main build
set -e
name=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)/tx-fast-hydrology_amd
L=$R/tx_fast_hydrology_amd/lib
mkdir -p $L/exp/obj_$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function "$@" -I $R/../include -I $R/csrc -c -o $L/exp/obj_$name/flow.hip.o ${SRC:-$R/csrc/flow.hip}
objs=$(ls $L/obj/*.o | grep -v flow.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $L/exp/lib_$name.so $objs $L/exp/obj_$name/flow.hip.o -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -pthread
echo built $name

#!/bin/bash
# A/B variant of the library: rebuild one kernel TU with extra -D flags and link it with the
# product's other objects into picotcp_amd/ab/libpicocsum_<name>.so (scripts/gpu_ab.sh A=<name>).
#   [SRC=<other source of the TU>] scripts/ab_build.sh <name> <tu: frag|raw|sorted_m0..3> -DFLAG=V ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; TU=$2; shift 2
make -s -j8 -C $R/picotcp_amd/csrc
B=$R/build/csrc; H=$R/picotcp_amd/csrc
mkdir -p $R/picotcp_amd/ab $B/ab
case $TU in
  sorted_m*) SRC=$H/pico_csum_k_sorted.hip; EXTRA=-DSORTED_MODE=${TU#sorted_m}; OBJ=$B/k_$TU.o ;;
  *) SRC=${SRC:-$H/pico_csum_k_$TU.hip}; EXTRA=; OBJ=$B/pico_csum_k_$TU.o ;;
esac
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I$R/include $EXTRA "$@" -c $SRC -o $B/ab/$NAME.o
OBJS=$(ls $B/pico_csum_k_raw.o $B/k_sorted_m?.o $B/pico_csum_k_frag.o $B/pico_csum.o | grep -v "^$OBJ\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/picotcp_amd/ab/libpicocsum_$NAME.so $OBJS $B/ab/$NAME.o \
    -Wl,--no-undefined -Wl,-soname,libpicocsum.so
echo "picotcp_amd/ab/libpicocsum_$NAME.so"

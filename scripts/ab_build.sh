#!/bin/bash
# A/B variant of the library: rebuild one kernel TU with extra -D flags and link it with the
# product's other objects into ablib/libpicocsum_<name>.so (scripts/gpu_ab.sh A=<name>).
#   [SRC=<other source of the TU>] scripts/ab_build.sh <name> <tu: frag|raw|sorted_m0..3|sorted_fused> -DFLAG=V ...
# sorted_fused: the sorted TU's fused modes 1-3 (the stream paths) from SRC, mode 0 from the product.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; TU=$2; shift 2
make -s -j8 -C $R/picotcp_amd/csrc
B=$R/build/csrc; H=$R/picotcp_amd/csrc
mkdir -p $R/ablib $B/ab
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I$R/include -I$R/picotcp_amd/csrc"
case $TU in
  sorted_fused)
    SRC=${SRC:-$H/pico_csum_k_sorted.hip}
    for m in 1 2 3; do $HIPCC -DSORTED_MODE=$m "$@" -c $SRC -o $B/ab/${NAME}_m$m.o & done; wait
    OBJS="$B/pico_csum_k_raw.o $B/k_sorted_m0.o $B/pico_csum_k_frag.o $B/pico_csum.o $B/ab/${NAME}_m1.o $B/ab/${NAME}_m2.o $B/ab/${NAME}_m3.o" ;;
  sorted_m*) SRC=${SRC:-$H/pico_csum_k_sorted.hip}; EXTRA=-DSORTED_MODE=${TU#sorted_m}; OBJ=$B/k_$TU.o ;;
  *) SRC=${SRC:-$H/pico_csum_k_$TU.hip}; EXTRA=; OBJ=$B/pico_csum_k_$TU.o ;;
esac
if [ $TU != sorted_fused ]; then
  $HIPCC $EXTRA "$@" -c $SRC -o $B/ab/$NAME.o
  OBJS="$(ls $B/pico_csum_k_raw.o $B/k_sorted_m?.o $B/pico_csum_k_frag.o $B/pico_csum.o | grep -v "^$OBJ\$") $B/ab/$NAME.o"
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/ablib/libpicocsum_$NAME.so $OBJS \
    -Wl,--no-undefined -Wl,-soname,libpicocsum.so
echo "ablib/libpicocsum_$NAME.so"

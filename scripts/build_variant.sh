# Variant library for A/B runs: the in-tree objects, with the listed translation units rebuilt
# under DEFS.  usage: bash scripts/build_variant.sh NAME "DEFS" tu1 [tu2 ...]  -> abx/lib_NAME.so
# (abx/: the libraries of the A/B session at hand; delete them after it, ab/ is gpurun-ignored)
set -e
cd "$(dirname "$0")/../tts-3_amd"
name=$1; defs=$2; shift 2
V=build_v_$name
rm -rf $V && mkdir -p $V ../abx && cp build/*.o $V/
for tu in "$@"; do
  extra=""
  case $tu in kernels_conv_wino|kernels_resblock|kernels_resblock2_*|kernels_convT_res|kernels_conv_split_h3|kernels_conv_split_b1|kernels_conv_split_x6|kernels_glow_wn) extra=-fno-slp-vectorize;; esac
  case $tu in kernels_conv*|kernels_resblock*) extra="$extra -Xarch_device -fno-honor-nans";; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc -Wall -Wno-unused-function $extra $defs -c csrc/$tu.hip -o $V/$tu.hip.o &
done
wait
printf 'extern "C" const char* tts_build_info(void) { return "target=gfx950 src=variant defs=%s"; }\n' "$(echo $defs | tr ' ' ',')" > $V/build_info.cpp
/opt/rocm/bin/hipcc -O2 -fPIC -x c++ -c $V/build_info.cpp -o $V/build_info.o
objs=$(ls build/*.o | sed "s#^build/#$V/#")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-soname,libtts_mi355x.so -Wl,--no-undefined $objs -o ../abx/lib_$name.so
rm -rf $V
echo "abx/lib_$name.so"

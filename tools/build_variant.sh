# Build a compile-time variant of libpinsage_hip.so: tools/build_variant.sh NAME FILE.hip "-DMACRO=..."
# -> variants/NAME/libpinsage_hip.so (PINSAGE_LIB=... selects it; A/B only)
set -e
name=$1; src=$2; flags=$3
cd "$(dirname "$0")/../gcn-song-embeddings_amd/csrc"
out=../../variants/$name; mkdir -p $out/obj
base=$(basename $src .hip)
/opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function $flags -c $src -o $out/obj/$base.o
objs=""
for o in build/*.o; do [ "$(basename $o)" = "$base.o" ] && objs="$objs $out/obj/$base.o" || objs="$objs $o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libpinsage_hip.so $objs -lpthread
echo built $out/libpinsage_hip.so

# build_variant_lib.sh NAME "-DFLAG=V ..." [SRC] : libthk.so with csrc/SRC.hip (default flash_attn) compiled
# under extra defines, linked with the other in-tree objects, written to ab_libs/NAME.so (for scripts/lib_ab.py)
set -e
cd "$(dirname "$0")/.."
python -m tensorhive_fixed_amd.ops.build >/dev/null
B=tensorhive_fixed_amd/ops/_build
SRC=${3:-flash_attn}
mkdir -p ab_libs /tmp/thk_variant
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-result \
  $(grep -m1 '^// th-build-flags:' tensorhive_fixed_amd/ops/csrc/$SRC.hip | cut -d: -f2) $2 \
  -I tensorhive_fixed_amd/ops/csrc -c tensorhive_fixed_amd/ops/csrc/$SRC.hip -o /tmp/thk_variant/$1.o 2>/dev/null
objs=$(ls $B/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs /tmp/thk_variant/$1.o -o ab_libs/$1.so
echo "built ab_libs/$1.so ($2)"

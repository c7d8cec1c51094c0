# Build A/B variants of the engine (compile-time toggles) into ponyc_amd/variants/.
set -e
cd "$(dirname "$0")/.."
OUT=ponyc_amd/variants
mkdir -p $OUT
b() { name=$1; shift; /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" -o $OUT/lib_$name.so ponyc_amd/csrc/engine.hip -lrccl & }
for v in "$@"; do
  case $v in
    base) b base ;;
    *) echo "unknown variant $v"; exit 1 ;;
  esac
done
wait
ls -la $OUT

# Build A/B variants of the engine (compile-time toggles) into ponyc_amd/variants/
# (objects under ponyc_amd/build/lib_<name>/; the units build in parallel).
set -e
cd "$(dirname "$0")/.."
OUT=ponyc_amd/variants
mkdir -p $OUT
b() {
  name=$1; shift
  python3 -c "import sys; from ponyc_amd import build as b; b.build(defines=sys.argv[2:], out=sys.argv[1])" \
    $OUT/lib_$name.so "$@"
}
for v in "$@"; do
  case $v in
    base) b base ;;
    # single-table (pinger) experiment builds: ~30 s instead of ~3 min
    p512) b p512 -DGPA_STEP_ONLY=2 ;;
    # single-table det / storm builds (the general handler path)
    d3) b d3 -DGPA_STEP_ONLY=3 ;;
    s8) b s8 -DGPA_STEP_ONLY=8 ;;
    # storm with 4096-actor zones (1024-thread workgroups, one per CU): runs twice as long
    s8z12) b s8z12 -DGPA_STEP_ONLY=8 -DGPA_ZONE_BITS=12 -DGPA_ZONE_THREADS=1024 -DGPA_IDX_CAP=24576 -DGPA_TILE=7168 ;;
    d3z12) b d3z12 -DGPA_STEP_ONLY=3 -DGPA_ZONE_BITS=12 -DGPA_ZONE_THREADS=1024 -DGPA_IDX_CAP=24576 -DGPA_TILE=7168 ;;
    p1024) b p1024 -DGPA_STEP_ONLY=2 -DGPA_ZONE_THREADS=1024 ;;
    z12a) b z12a -DGPA_ZONE_BITS=12 -DGPA_ZONE_THREADS=1024 -DGPA_IDX_CAP=24576 -DGPA_TILE=7168 ;;
    z12b) b z12b -DGPA_ZONE_BITS=12 -DGPA_ZONE_THREADS=1024 -DGPA_IDX_CAP=32768 -DGPA_TILE=8192 ;;
    *) echo "unknown variant $v"; exit 1 ;;
  esac
done
ls -la $OUT

#!/bin/bash
# A/B of config 5's rank-0 slice (8 ranks, emulated) over layouts / knobs of the dev build.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT" || exit 1
DEV=$ROOT/build/dev/libsparsematrix_amd.so
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload config5 --emulate-world ${EMU:-8} --steps 10 --warmup 2 --replays 3 --no-cpu > "$OUT/c5_$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/c5_$name.log"; return 1; }
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']; print(f\"{sys.argv[2]:24s} {r['kernel_ms']*1e3:9.1f} us  {r['layout']:8s} frac {r['frac']}\")" "$OUT/c5_$name.log" "$name"
}
eval "${VARIANTS:-true}"

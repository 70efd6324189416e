#!/bin/bash
# Round-4 GPU session driver: each step under its own time limit; a test failure (exit 1) is
# recorded and the session goes on, anything else (a fault, an abort, a time limit) ends it.
#   tools/gpu_steps.sh TAG 'step' ['step' ...]     e.g. tools/gpu_steps.sh r4a "tests tests/test_gpu_raw.py" bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {   # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/steps.txt" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)" >&2; exit $rc; fi
  return 0
}
for step in "$@"; do
  set -- $step
  kind=$1; shift
  case $kind in
    tests) run "pytest_$(echo "$*" | tr -c 'a-zA-Z0-9' '_' | cut -c1-60)" 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "$@" ;;
    alltests) run pytest_all 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run "bench_$(echo "$*" | tr -c 'a-zA-Z0-9' '_' | cut -c1-60)" 600 python -u bench.py "$@" ;;
    py) name=$1; shift; run "$name" 600 python -u "$@" ;;
    *) echo "unknown step $kind" >&2; exit 2 ;;
  esac
done
echo "all steps done" >&2

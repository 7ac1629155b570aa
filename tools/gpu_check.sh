#!/bin/bash
# One parameterised GPU-box script (replaces the per-call lease scripts of round 1).
#   tools/gpu_check.sh tests      full `pytest -m gpu` tier
#   tools/gpu_check.sh smoke      __graft_entry__.smoke()
#   tools/gpu_check.sh bench      headline bench.py (driver contract defaults + op backends)
#   tools/gpu_check.sh prof       rocprofv3 --kernel-trace --stats of a short bench + markdown summary
#   tools/gpu_check.sh all        tests, smoke, bench (round-end style)
# Each GPU step runs under its own timeout; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
tag="${TAG:-run}"
step() {  # step <secs> <name> <cmd...>
  local secs=$1 name=$2; shift 2
  echo "=== [$name] $(date +%T)"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_${name}.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc $(date +%T)"; tail -n 15 "gpurun_out/${tag}_${name}.log"
  return $rc
}
tests() { step 900 pytest python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread; }
smoke() { step 300 smoke python -u -c "import __graft_entry__ as g; g.smoke()"; }
bench() { step 600 bench python -u bench.py ${BENCH_ARGS:---profile-ops}; }
prof() {
  step 600 prof rocprofv3 --kernel-trace --stats -d /tmp/prof_${tag} -o run -- \
      python3 bench.py --steps ${PROF_STEPS:-2} --warmup 1 ${BENCH_ARGS:-} || return $?
  db=$(find /tmp/prof_${tag} -name "*results.db" | head -n1)
  [ -n "$db" ] && python -m comfy_gen_server_amd.tools.rocprof_summary "$db" "gpurun_out/${tag}_prof.md" --top 60 ${PROF_TAIL:+--tail-s $PROF_TAIL}
  return 0
}
for what in "$@"; do
  case "$what" in
    all) tests && smoke && bench || exit $? ;;
    tests|smoke|bench|prof) $what || exit $? ;;
    *) echo "unknown step $what"; exit 2 ;;
  esac
done

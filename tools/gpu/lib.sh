# shared helper of the tools/gpu call scripts: step <name> <timeout s> <cmd...>
# runs one GPU step under its own time limit with stdout/stderr in $O/<name>.out/.err.  An ordinary
# failure (exit 1, e.g. a Python exception) is recorded and the script goes on; a time limit, abort,
# segfault, any signal death (exit >= 124) or a reported GPU memory fault ends the script: nothing more
# touches the GPU.
step() {
  local name=$1 secs=$2
  shift 2
  local rc=0
  timeout -k 10 "$secs" "$@" > "$O/$name.out" 2> "$O/$name.err" || rc=$?
  echo "$name rc=$rc" | tee -a "$O/steps.txt"
  # a GPU memory fault surfaces as a Python exception (rc 1): treat it like a crash
  if grep -qE "illegal memory access|MEMORY_APERTURE_VIOLATION|Memory access fault|HSA_STATUS_ERROR" "$O/$name.out" "$O/$name.err" 2>/dev/null; then
    echo "stopping after $name (GPU fault reported)" | tee -a "$O/steps.txt"
    exit 97
  fi
  if [ "$rc" -ge 124 ]; then
    echo "stopping after $name (rc=$rc)" | tee -a "$O/steps.txt"
    exit "$rc"
  fi
}

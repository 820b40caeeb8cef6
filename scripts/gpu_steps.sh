# Run GPU steps on the box, each under its own time limit (timeout -k 10),
# stopping at the first failure; every step's output goes to $OUT/<name>.log.
# usage: OUT=gpurun_out/<tag> bash scripts/gpu_steps.sh 'name|seconds|command' ...
# Steps named pytest* may exit 1 (test failures) and the run continues.
export TMPDIR=/tmp
O=${OUT:-gpurun_out/steps}
mkdir -p "$O"
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "[$(date +%T)] $name: $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "$O/$name.log" 2>&1; rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then
    case $name in pytest*) [ $rc -eq 1 ] && continue ;; esac
    exit $rc
  fi
done
echo done

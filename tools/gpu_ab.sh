# A/B of library builds and switches in ONE box session (boxes differ by ~10%):
#   bash tools/gpu_ab.sh <tag> "<label>:<env assignments or ->:<bench args>" ...
# each arm: NAME=label, optional MDEMI_LIB=tools/study/<x>/libmdemi.so etc. in the env part
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=$1; shift
for arm in "$@"; do
  label=${arm%%:*}; rest=${arm#*:}; envs=${rest%%:*}; args=${rest#*:}
  [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 300 python -u bench.py $args > gpurun_out/ab_${tag}_$label.log 2>&1 || { echo "arm $label failed"; tail -5 gpurun_out/ab_${tag}_$label.log; exit 1; }
  grep "^{\"metric" gpurun_out/ab_${tag}_$label.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(\"$label\", d[\"value\"], d[\"ms_per_step\"])"
done

# chain probe sweep (tools/tchain_probe*, make tchain-probe): tools/probe_r5u.sh TAG BIN [BIN ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=$1
shift
for b in "$@"; do
  for p in 0 1 2 3; do
    for r in 24874 65536; do
      timeout -k 5 60 tools/$b $p $r 20 >> gpurun_out/${tag}_probe.log 2>&1 || { echo "FAIL $b $p $r"; exit 1; }
      echo "$b $(tail -1 gpurun_out/${tag}_probe.log)"
    done
  done
done

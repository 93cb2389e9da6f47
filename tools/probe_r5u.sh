set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in tchain_probe tchain_probe_nb4 tchain_probe_exp1 tchain_probe_exp2; do
  for p in 0 1 2 3; do
    for r in 24874 65536; do
      timeout -k 5 60 tools/$b $p $r 20 >> gpurun_out/r5u_probe.log 2>&1 || { echo "FAIL $b $p $r"; exit 1; }
      echo "$b $(tail -1 gpurun_out/r5u_probe.log)"
    done
  done
done

cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --shard-steps 0 --steps 4000 --warmup 300 --spec-rounds $r > gpurun_out/spec_$r.log 2>&1 || exit 1
  echo "rounds=$r: $(tail -1 gpurun_out/spec_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["speculation"]; print(d["value"], s["steps"], s["host_round_steps"], s["rounds"])')"
done

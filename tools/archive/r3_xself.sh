#!/bin/bash
# One rank, N=512 fp64 fma: the periodic x wrap sent through RCCL to the rank itself
# (--x-self-transport; RCCL send/recv on the comm stream) with overlap on / off, against the
# fused local wrap. Best of 3 solves (after 1 warm-up), 2 rounds.
cd "$(dirname "$0")/.."
port=29611
run() {
  port=$((port + 1))
  timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $port tools/dist_solve.py --backend hip --transport rccl -- 512 1 pi pi pi 1 100 --math fma \
      --repeat 3 --warmup 1 --format none --quiet "$@" 2>/dev/null | grep '^RESULT' | cut -c8- \
    | python3 -c "import sys,json; r=json.loads(sys.stdin.read()); print(round(r['mpts_per_s_best']), r['kernel'], 'overlap', r['overlap'], 'exch_ms', round(r['exchange_ms'],1), 'comm_ms', round(r['comm_ms'],1), 'linf', '%.9g' % r['max_abs'][-1])"
}
for rep in 1 2; do
  echo -n "rep=$rep fused wrap: "; run || exit 1
  echo -n "rep=$rep x-self-transport overlap off: "; run --x-self-transport --overlap off || exit 1
  echo -n "rep=$rep x-self-transport overlap on: "; run --x-self-transport --overlap on || exit 1
done

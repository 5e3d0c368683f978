#!/bin/bash
# C5 at 30M records: where pv_process_host's time goes (ingest split), and a rocprofv3 trace of it
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r4_w; mkdir -p $O
timeout -k 10 300 python3 -u bench.py --config 5 --stream-records 30000000 --steps 1 --warmup 1 > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
tail -1 $O/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['ingest_ms'])"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o k -- python3 $R/bench.py --config 5 --stream-records 30000000 --steps 1 --warmup 0 > $O/prof.log 2>&1) || { tail -5 $O/prof.log; exit 1; }
python3 tools/kstats.py $O/prof | cut -c1-400

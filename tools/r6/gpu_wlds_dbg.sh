#!/bin/bash
# where the weight-resident kernel's time goes: replay of the 3-tap convs with the diagnostic switches
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r6wdbg}; mkdir -p $O; cd $R
grep '"ntaps": 3' profiles/r05/gemm_log_parity.jsonl | grep '"M": 9600, "N": 256' > $O/log3.jsonl
for d in 0 1 2 3; do
  MTTS_WLDS_DBG=$d timeout -k 10 200 python -u tools/r5/gemm_replay.py $O/log3.jsonl --only-bf16 --cfgs=-1,64 --out $O/replay_dbg$d.jsonl > $O/replay_dbg$d.log 2>&1 || exit 1
  echo "dbg=$d"; python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    if 'res' in d: print(d['M'],d['N'],d['K'],d['flags'],d['res']['-1']['us'],d['res']['64'].get('us'))
" $O/replay_dbg$d.jsonl
done

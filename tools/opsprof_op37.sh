#!/bin/bash
# ops-prof's multi-tune sweep over the reference's 42-op 3x3 list (test/test_cmds.xml:110's invocation,
# the tunes of tests/test_gpu_opsprof.py), every run line kept: which tunes miss op 37's stored digest
# (the documented outlier) and by how much (worst rd/tol per tune)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=${1:-gpurun_out/opsprof_op37.log}
python3 -c "import json; print(''.join(e['op'] + '\n' for e in json.load(open('tests/golden/ops-prof-conv-3x3-cudnn-boda.json'))), end='')" \
  > gpurun_out/op37_ops.txt
T="(kg=(use_be=hip,cfg=ref64),tab=(use_be=hip),dm=(cfg=dm3w16x64c8),tile=(cfg=128x128x32),gvs=(cfg=gvs64x32w8),"
T="${T}wx43=(cfg=wx43s12),wx23=(cfg=wx23s6),wx25=(cfg=wx25s6),wgi=(cfg=wgi128x32),wgl=(cfg=wgl128x32))"
timeout -k 10 600 boda-1_amd/bin/boda_hip_ops_prof --ops-fn=gpurun_out/op37_ops.txt \
  --wisdom-in-fn=tests/golden/wis/ops-prof-conv-3x3-cudnn-boda.wis --op-tunes="$T" --kg-tune-tag=kg \
  --gen-data-mode=5 --write-runs=1 --live-mrd-toler=2e-3 --wisdom-out-fn=gpurun_out/op37_out.wis > "$out" 2>&1
echo "ops-prof rc=$?" >> "$out"
grep -E "op_ix=37 " "$out" | head -40

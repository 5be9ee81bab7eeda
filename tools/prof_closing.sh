#!/bin/bash
# Closing evidence: rocprofv3 kernel trace + stats of the exact default bench command, reconciled with its bench line.
set -o pipefail
bash tools/prof_default_cmd.sh || exit 1
python3 tools/reconcile_trace.py gpurun_out/defcmd/kernel_trace.csv gpurun_out/defcmd/bench.json gpurun_out/defcmd/reconcile.json || exit 1
cat gpurun_out/defcmd/reconcile.json
head -5 gpurun_out/defcmd/kernel_stats.csv | cut -c1-200
rm -f gpurun_out/defcmd/kernel_trace.csv

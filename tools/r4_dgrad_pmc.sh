#!/bin/bash
# PMC passes over the isolated layer-1 DGRAD+BNR shape (tools/dgrad_pmc.py): bytes fetched / written
# against the ideal, VMEM / LDS / VALU instruction counts, wave cycles and wait cycles.
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/pmc; cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python -u $R/tools/dgrad_pmc.py > $R/gpurun_out/pmc/time.txt 2>&1 || exit 1
FOLD=1 timeout -k 10 120 python -u $R/tools/dgrad_pmc.py >> $R/gpurun_out/pmc/time.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc/p1 -o run -- python $R/tools/dgrad_pmc.py > $R/gpurun_out/pmc/p1.log 2>&1 || { tail -20 $R/gpurun_out/pmc/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $R/gpurun_out/pmc/p2 -o run -- python $R/tools/dgrad_pmc.py > $R/gpurun_out/pmc/p2.log 2>&1 || { tail -20 $R/gpurun_out/pmc/p2.log; exit 1; }
find $R/gpurun_out/pmc -name "*.csv" | head

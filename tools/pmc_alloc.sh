#!/bin/bash
# Memory-side counters of the headline kernel across allocations (tools/contig_probe.py rounds):
# local-DRAM vs all requests, UTCL2 busy, credit stalls.  One --pmc pass per counter group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PROBE_STEPS=3
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE \
  -d gpurun_out/pmc_a -o a --output-format csv -- python3 tools/contig_probe.py > gpurun_out/pmc_a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_GMI_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum \
  -d gpurun_out/pmc_b -o b --output-format csv -- python3 tools/contig_probe.py > gpurun_out/pmc_b.log 2>&1

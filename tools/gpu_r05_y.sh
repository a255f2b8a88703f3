#!/bin/bash
# round 5: steady-state step time vs the same steps queued behind a spin
# kernel (host certainly ahead): is there host-induced GPU idle unprofiled?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 240 python3 -u tools/host_lead_probe.py > $OUT/r05_y_host_lead.txt 2>&1 || exit $?
cat $OUT/r05_y_host_lead.txt | grep -v amdgpu.ids | head -4

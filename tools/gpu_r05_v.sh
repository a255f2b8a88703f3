#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_lead_probe.py > gpurun_out/r05_host_lead.txt 2>&1 || exit $?
head -60 gpurun_out/r05_host_lead.txt | cut -c1-220

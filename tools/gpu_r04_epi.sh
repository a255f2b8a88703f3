# GEMM epilogue-schedule experiment (tools/gemm_epi.hip)
mkdir -p gpurun_out
timeout -k 10 300 tools/bin/gemm_epi 204632 9 > gpurun_out/r04_gemm_epi.txt 2>&1

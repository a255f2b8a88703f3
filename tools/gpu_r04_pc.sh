# NT GEMM producer/consumer experiment (tools/gemm_pc.hip) at whole rounds
mkdir -p gpurun_out
timeout -k 10 120 tools/bin/gemm_pc 196608 9 > gpurun_out/r04_gemm_pc.txt 2>&1

# NT GEMM ablations on the pre-cleanup kernel (git HEAD~2 of round 4): the
# B-fragment DMA, the A DMA, the MFMAs + split removed (timing only)
mkdir -p gpurun_out
for n in base nob nomfma nomfma_nob noa base; do
  echo "== $n" >> gpurun_out/r04_gemm_ablate.txt
  GB_NOCHECK=1 timeout -k 10 120 tools/bin/gb_$n 204632 >> gpurun_out/r04_gemm_ablate.txt 2>&1 || exit $?
done

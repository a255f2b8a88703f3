# NT GEMM ablations that really remove the main loop's A or B DMAs (the
# round-2 flags sat in a branch the kernel no longer took): timing only
mkdir -p gpurun_out
for v in new2 noa nob new2 noa nob; do
  echo "== $v" >> gpurun_out/r04_nt_ablate.txt
  GB_NOCHECK=1 timeout -k 10 120 tools/bin/gemm_ab_$v 204632 7 >> gpurun_out/r04_nt_ablate.txt 2>&1 || exit $?
done

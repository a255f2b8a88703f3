# Weight-gradient kernel A/B on one lease (old / new binary alternated),
# the encoder's shapes and the CE backward's two products
mkdir -p gpurun_out
for v in old new2 old new2 old new2; do
  echo "== $v" >> gpurun_out/r04_tn_ab.txt
  timeout -k 10 120 tools/bin/gemm_ab_$v 204632 9 >> gpurun_out/r04_tn_ab.txt 2>&1 || exit $?
done

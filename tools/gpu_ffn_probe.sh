# A/B of the fused FeedForward activation GEMMs: ACT on 256 x 256 tiles
# (tile-end epilogue, default) vs 256 x 128 tiles (deferred epilogue)
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in "" datamining_recblr_amd/lib/ab_act4.so "" datamining_recblr_amd/lib/ab_act4.so; do
  RECBLR_LIB=$lib timeout -k 10 240 python -u tools/ffn_act_probe.py >> gpurun_out/r03_ffn_probe2.txt 2>&1 || exit $?
done

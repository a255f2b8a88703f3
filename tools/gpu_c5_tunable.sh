# configs[4] step with PyTorch TunableOp (hipBLASLt / rocBLAS solution search
# for the bf16 projection GEMMs) against the default heuristic
mkdir -p gpurun_out
timeout -k 10 200 python tools/c5_step.py 4 > gpurun_out/c5_default.txt 2>&1 || exit $?
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=0 \
  PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_c5.csv \
  timeout -k 10 500 python tools/c5_step.py 4 > gpurun_out/c5_tune.txt 2>&1 || exit $?
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 \
  PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_c5.csv \
  timeout -k 10 200 python tools/c5_step.py 4 > gpurun_out/c5_tuned.txt 2>&1

set -u
mkdir -p gpurun_out/r7a
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -s -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  "tests/test_gpu_model.py::test_vit_base_full_depth_fp32_vs_fp64" \
  "tests/test_gpu_dropin.py::test_vit_base_depth12_teacher_forced_blocks_bf16" \
  "tests/test_gpu_dropin.py::test_vit_base_full_depth_bf16_train_properties" \
  "tests/test_gpu_dropin.py::test_c2_full_shape_bf16_train_vs_oracle" \
  tests/test_gpu_kernels.py -k "attention_fwd_bwd or tiled_kernels_any_grid or full_depth or teacher or c2_full" \
  > gpurun_out/r7a/new.log 2>&1
echo "new rc=$?" >> gpurun_out/r7a/status.txt

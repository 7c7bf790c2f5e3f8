set -u
OUT=gpurun_out/r3d; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_model.py tests/test_image_pipeline.py -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; echo "tests rc=$?"
grep -E "PASS|FAIL|ERROR|worst" $OUT/tests.log | tail -50

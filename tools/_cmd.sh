timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || exit $?
for sc in 0 1; do timeout -k 10 300 python3 tools/tune.py --scene $sc --spp 128 --rounds 4 --configs "RT_JIT_FASTDIV=0,RT_JIT_FASTDIV=1,RT_JIT_SHARE_RCP=1" > gpurun_out/tune_s$sc.log 2>&1 || exit $?; done

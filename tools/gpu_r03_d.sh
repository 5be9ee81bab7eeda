# after the short-block rocBLAS dispatch: the India exp driver, config 3, the Hessian driver, then tests
set -e
O=gpurun_out/r03d; mkdir -p $O





timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log

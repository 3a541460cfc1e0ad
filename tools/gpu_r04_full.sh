# Round-4: the full-size parity tests (numbers printed) + the new Bayes VAE / materialise tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
O=gpurun_out/r04
timeout -k 10 1100 python -u -m pytest tests/test_north_star.py tests/test_full_size.py tests/test_e2e_vae.py tests/test_materialize.py -v -s -m gpu --timeout 1000 --timeout-method thread > $O/pytest_full2.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest_full2.log | tail -3
exit $rc

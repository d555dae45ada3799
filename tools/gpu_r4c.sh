# round-4 check: k_hot_bx draws unchanged (winners of the previous commit's
# kernels, both with the degree-2 exp), near-tie agreement with the degree-2
# exp (variant) and the degree-3 exp (product), the whole GPU suite, bench
set -o pipefail
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 200 python -u tools/ab_winners.py $O/prod.npz > $O/ab.log 2>&1 || exit 1
HYPEROPT_AMD_VARIANT=tools/var_r4khot.so timeout -k 10 200 python -u tools/ab_winners.py $O/khot.npz >> $O/ab.log 2>&1 || exit 1
HYPEROPT_AMD_VARIANT=tools/var_r4base.so timeout -k 10 200 python -u tools/ab_winners.py $O/base.npz >> $O/ab.log 2>&1 || exit 1
echo "== base vs khot (k_hot_bx rewrite: must be identical)" >> $O/ab.log
python tools/ab_winners.py --compare $O/base.npz $O/khot.npz >> $O/ab.log 2>&1
echo "== khot vs prod (degree-3 exp)" >> $O/ab.log
python tools/ab_winners.py --compare $O/khot.npz $O/prod.npz >> $O/ab.log 2>&1
mkdir -p $O/deg2
NEAR_TIE_OUT=$O/deg2 HYPEROPT_AMD_VARIANT=tools/var_r4khot.so timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_near_tie_agreement.py > $O/nt_deg2.log 2>&1
mkdir -p $O/deg3
NEAR_TIE_OUT=$O/deg3 timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1

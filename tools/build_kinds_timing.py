"""Device posterior-build kernel times per history shape (run under
rocprofv3 --kernel-trace): continuous-only (Hartmann-6 labels) vs the mixed
config-3 space (with categorical labels), both at N = 10k.

    rocprofv3 --kernel-trace -d out -o run --output-format csv -- \
        python tools/build_kinds_timing.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch  # noqa: F401  (one HIP runtime)
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import hartmann_history, mixed_history
    eng = Engine(0, 'f64')
    for name, hist in (('hartmann6_10k', hartmann_history(10000, seed=0)),
                       ('mixed32_10k', mixed_history(32, 10000, seed=0))):
        inp = hist.device_inputs()
        for _ in range(4):
            eng.build_posterior(*inp, gamma=0.25, prior_weight=1.0)
        print(name, 'kernels ms', eng.last_build_ms(), flush=True)
    eng.close()


if __name__ == '__main__':
    main()

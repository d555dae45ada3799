"""Host-side profile of config 3's fmin step (experiment): the step run as
bench.py runs it (FminLoop.advance with the round inside), cProfile over
`steps` steps, the top functions by own and cumulative time.
    python tools/host_profile.py [steps]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch  # noqa: F401  (the HIP runtime first)
    from hyperopt_amd.engine import Engine
    from hyperopt_amd.workloads import FminLoop, mixed_history
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    N0, C = 10000, 1 << 24
    hist = mixed_history(32, N0 + steps + 8, seed=0)
    eng = Engine(0, 'f64')
    loop = FminLoop(hist)
    loop.advance(eng, N0)

    def step(i):
        rc = lambda: eng.suggest(seed=1234 + i, n_candidates=C, round=i)  # noqa: E731
        return loop.advance(eng, N0 + 1 + i, n_candidates=C, n_rounds=1, round_call=rc)
    for i in range(3):
        step(i)
    t0 = time.perf_counter()
    pr = cProfile.Profile()
    pr.enable()
    for i in range(3, 3 + steps):
        step(i)
    pr.disable()
    dt = (time.perf_counter() - t0) / steps
    print('ms per step (profiled): %.3f' % (1e3 * dt))
    st = pstats.Stats(pr)
    st.sort_stats('tottime').print_stats(25)
    st.sort_stats('cumulative').print_stats(30)
    eng.close()


if __name__ == '__main__':
    main()

"""In-tree build of the native pieces (no JIT cache, so the .so files travel
with the repository snapshot to the GPU box).

    python -m hyperopt_amd._build
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = 'gfx950'

SOURCES = [os.path.join(HERE, 'csrc', 'tpe_engine.hip'), os.path.join(HERE, 'csrc', 'tpe_build.hip')]
DEPS = SOURCES + [os.path.join(HERE, 'csrc', 'tpe_device.h'),
                  os.path.join(HERE, 'csrc', 'tpe_ctx.h'),
                  os.path.join(HERE, 'csrc', 'tpe_exp_table.h'),
                  os.path.join(REPO, 'include', 'hyperopt_tpe.h')]
TARGET = os.path.join(HERE, 'libhyperopt_tpe.so')

FLAGS = ['--offload-arch=' + ARCH, '-O3', '-std=c++17', '-fPIC', '-shared',
         '-Wall', '-Wno-unused-function', '-I' + os.path.join(REPO, 'include')]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_engine(force=False, verbose=True):
    if not force and not _stale(TARGET, DEPS):
        return TARGET
    cmd = [HIPCC] + FLAGS + ['-o', TARGET] + SOURCES
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.check_call(cmd)
    return TARGET


def build_oracle(force=False, verbose=True):
    """The C restatement of the scorer lives under oracle/ (test infra)."""
    mk = os.path.join(REPO, 'oracle', 'Makefile')
    if os.path.exists(mk):
        subprocess.check_call(['make', '-s', '-C', os.path.join(REPO, 'oracle')] +
                              (['-B'] if force else []))


def main(argv):
    force = '--force' in argv
    build_engine(force=force)
    build_oracle(force=force)


if __name__ == '__main__':
    main(sys.argv[1:])

"""In-tree build of the gfx950 engine library (no JIT cache, so the .so
travels with the repository snapshot to the GPU box).

    python -m hyperopt_amd._build [--force]

The library is stamped with a hash of the sources it was compiled from
(`tpe_source_hash()`); `_lib.load()` recomputes the hash from the sources in
the tree and refuses a library built from anything else, so a stale `.so`
can never run in place of HEAD's code.
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = 'gfx950'

SOURCES = [os.path.join(HERE, 'csrc', 'tpe_engine.hip'),
           os.path.join(HERE, 'csrc', 'tpe_build.hip'),
           os.path.join(HERE, 'csrc', 'tpe_multi.hip'),
           os.path.join(HERE, 'csrc', 'tpe_window.hip'),
           os.path.join(HERE, 'csrc', 'tpe_expand.hip'),
           os.path.join(HERE, 'csrc', 'tpe_share.hip')]
DEPS = SOURCES + [os.path.join(HERE, 'csrc', 'tpe_device.h'),
                  os.path.join(HERE, 'csrc', 'tpe_ctx.h'),
                  os.path.join(HERE, 'csrc', 'tpe_exp_table.h'),
                  os.path.join(REPO, 'include', 'hyperopt_tpe.h')]
TARGET = os.path.join(HERE, 'libhyperopt_tpe.so')

FLAGS = ['--offload-arch=' + ARCH, '-O3', '-std=c++17', '-fPIC', '-shared',
         '-Wall', '-Wno-unused-function', '-I' + os.path.join(REPO, 'include')]


def source_hash(deps=DEPS):
    """sha256 (first 16 hex digits) over the build inputs and the flags."""
    h = hashlib.sha256()
    for d in deps:
        h.update(os.path.basename(d).encode())
        with open(d, 'rb') as f:
            h.update(f.read())
    # flags without the tree's absolute location (the GPU box unpacks it elsewhere)
    h.update(' '.join(f for f in FLAGS if not f.startswith('-I')).encode())
    return h.hexdigest()[:16]


def built_hash(target=TARGET):
    """The hash stamped into an existing library (None if absent/unstamped);
    read from the file's bytes, without loading it."""
    if not os.path.exists(target):
        return None
    with open(target, 'rb') as f:
        data = f.read()
    tag = b'TPE_SOURCE_HASH='
    i = data.find(tag)
    if i < 0:
        return None
    return data[i + len(tag):i + len(tag) + 16].decode('ascii', 'replace')


def build_engine(force=False, verbose=True):
    """Compile every source to an object in parallel (each carries its own
    gfx950 code object), then link the shared library."""
    import tempfile
    want = source_hash()
    if not force and built_hash(TARGET) == want:
        return TARGET
    flags = FLAGS + ['-DTPE_SOURCE_HASH="%s"' % want]
    with tempfile.TemporaryDirectory(prefix='tpe_build_') as tmp:
        objs, procs = [], []
        for src in SOURCES:
            obj = os.path.join(tmp, os.path.basename(src) + '.o')
            cmd = [HIPCC] + [f for f in flags if f != '-shared'] + ['-c', '-o', obj, src]
            if verbose:
                print(' '.join(cmd), flush=True)
            procs.append(subprocess.Popen(cmd))
            objs.append(obj)
        bad = [src for src, p in zip(SOURCES, procs) if p.wait() != 0]
        if bad:
            raise RuntimeError('hipcc failed on %s' % ', '.join(os.path.basename(b) for b in bad))
        cmd = [HIPCC] + flags + ['-o', TARGET] + objs
        if verbose:
            print(' '.join(cmd), flush=True)
        subprocess.check_call(cmd)
    got = built_hash(TARGET)
    if got != want:
        raise RuntimeError('built library carries hash %r, expected %r' % (got, want))
    return TARGET


def main(argv):
    build_engine(force='--force' in argv)


if __name__ == '__main__':
    main(sys.argv[1:])

"""Build an engine variant with extra preprocessor definitions into
tools/var_<name>.so, stamped with the tree's own source hash so the loader
takes it when it is copied over hyperopt_amd/libhyperopt_tpe.so (timing
experiments only: tools/var_sweep.sh, tools/var_trace.sh).

    python tools/build_variant.py bm TPE_EXP_BM_CHEAP
    python tools/build_variant.py norej TPE_EXP_NO_REJECT
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hyperopt_amd import _build  # noqa: E402


def main(name, defs):
    base = _build.source_hash()          # the variant loads as the tree's own build
    _build.source_hash = lambda deps=None: base
    _build.FLAGS = _build.FLAGS + ['-D' + d for d in defs]
    _build.TARGET = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'var_%s.so' % name)
    try:
        _build.build_engine(force=True, verbose=False)
    except RuntimeError:   # (the post-build check reads the tree's own library)
        pass
    print('built', _build.TARGET)


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2:])

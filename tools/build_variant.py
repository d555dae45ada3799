"""Build a timing variant of the engine (experiments only) into
tools/var_<name>.so from a PATCHED COPY of the sources: the product sources
carry no experiment switches.  A variant is stamped 'v:<name>:' + a hash of
the patched sources, so the product loader refuses it unless the process
opts in explicitly with HYPEROPT_AMD_VARIANT=<path to the variant> (the
product library in hyperopt_amd/ is never overwritten).

    python tools/build_variant.py bm        # Box-Muller radius without its log and sqrt (not a normal draw)
    python tools/build_variant.py norej     # no truncation rejection (wrong samples)
    python tools/build_variant.py hot4 -DTPE_HOT_R=4   # a compile-time constant changed

    HYPEROPT_AMD_VARIANT=tools/var_bm.so python bench.py ...
"""
import hashlib
import os
import shutil
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
from hyperopt_amd import _build  # noqa: E402

# name -> [(file, old text, new text)]: result-changing timing experiments
PATCHES = {
    # the expansion index's cut: components left out below 2^-64 / 2^-48 of the
    # largest term instead of 2^-96 (narrower windows and fewer bins; the
    # screen's bound carries the skipped mass)
    'bxt64': [('tpe_device.h', 'constexpr double kBxT = 96.0;', 'constexpr double kBxT = 64.0;')],
    'bxt48': [('tpe_device.h', 'constexpr double kBxT = 96.0;', 'constexpr double kBxT = 48.0;')],
    # k_bx_table: ocml's fp64 exp (<= 1 ulp) instead of the 32 KB LDS table exp: no
    # table load per workgroup, no dependent LDS read per term, 5 workgroups per CU
    'bxexp': [('tpe_expand.hip', '    __shared__ double lds[kExpTabSize];   // the exp table, then the waves\' partial sums',
               '    __shared__ double lds[3 * kTabSums * 64];   // the waves\' partial sums'),
              ('tpe_expand.hip', '    load_exp_table(lds);\n    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;\n    const int b = b0 + lane, blast',
               '    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;\n    const int b = b0 + lane, blast'),
              ('tpe_expand.hip', 'const double e = exp_scaled(fmin(aj[q] * kExpScale, 0.0), lds);',
               'const double e = exp(fmin(aj[q], 0.0));')],
    # k_bx_table: the 15 powers of each component's Taylor argument as a tree
    # (y^2, y^4, y^8; depth ~5 instead of a 14-multiply chain)
    'bxtree': [('tpe_expand.hip',
                """#pragma unroll
            for (int n = 1; n < kBxP; ++n)
#pragma unroll
                for (int q = 0; q < kBxChains; ++q) {
                    t[q] *= y[q];
                    A[n] = fma(t[q], kInvFact[n], A[n]);
                }
#pragma unroll
            for (int q = 0; q < kBxChains; ++q) S3 += fabs(t[q] * y[q]);""",
                """#pragma unroll
            for (int q = 0; q < kBxChains; ++q) {
                const double y1 = y[q], y2 = y1 * y1, y4 = y2 * y2, y8 = y4 * y4;
                double p[kBxP + 1];
                p[1] = t[q] * y1;
                p[2] = t[q] * y2;
                p[4] = t[q] * y4;
                p[8] = t[q] * y8;
                p[3] = p[1] * y2;
                p[5] = p[1] * y4;
                p[6] = p[2] * y4;
                p[9] = p[1] * y8;
                p[10] = p[2] * y8;
                p[12] = p[4] * y8;
                p[7] = p[3] * y4;
                p[11] = p[3] * y8;
                p[13] = p[5] * y8;
                p[14] = p[6] * y8;
                p[15] = p[7] * y8;
#pragma unroll
                for (int n = 1; n < kBxP; ++n) A[n] = fma(p[n], kInvFact[n], A[n]);
                S3 += fabs(p[15]);
            }""")],
    # bins twice as wide (Taylor argument <= ~1) with 32 sub-bins each: measured slower (r5g)
    'sub32': [('tpe_device.h', 'constexpr int kBxSubBits = 4;', 'constexpr int kBxSubBits = 5;'),
              ('tpe_expand.hip', 'const double r_target = 0.25 / (kap * d0);',
               'const double r_target = 0.5 / (kap * d0); ')],
    # k_bx_table: the 15 powers of each component's Taylor argument as a tree
    # (y^2, y^4, y^8; depth ~5 instead of a 14-multiply chain)
    'bxtree': [('tpe_expand.hip',
                """#pragma unroll
            for (int n = 1; n < kBxP; ++n)
#pragma unroll
                for (int q = 0; q < kBxChains; ++q) {
                    t[q] *= y[q];
                    A[n] = fma(t[q], kInvFact[n], A[n]);
                }
#pragma unroll
            for (int q = 0; q < kBxChains; ++q) S3 += fabs(t[q] * y[q]);""",
                """#pragma unroll
            for (int q = 0; q < kBxChains; ++q) {
                const double y1 = y[q], y2 = y1 * y1, y4 = y2 * y2, y8 = y4 * y4;
                double p[kBxP + 1];
                p[1] = t[q] * y1;
                p[2] = t[q] * y2;
                p[4] = t[q] * y4;
                p[8] = t[q] * y8;
                p[3] = p[1] * y2;
                p[5] = p[1] * y4;
                p[6] = p[2] * y4;
                p[9] = p[1] * y8;
                p[10] = p[2] * y8;
                p[12] = p[4] * y8;
                p[7] = p[3] * y4;
                p[11] = p[3] * y8;
                p[13] = p[5] * y8;
                p[14] = p[6] * y8;
                p[15] = p[7] * y8;
#pragma unroll
                for (int n = 1; n < kBxP; ++n) A[n] = fma(p[n], kInvFact[n], A[n]);
                S3 += fabs(p[15]);
            }""")],
    # round 4's index geometry: bins half as wide (Taylor argument <= ~0.5), 16 sub-bins each
    'sub16': [('tpe_device.h', 'constexpr int kBxSubBits = 5;', 'constexpr int kBxSubBits = 4;'),
              ('tpe_expand.hip', 'const double r_target = 0.5 / (kap * d0); ',
               'const double r_target = 0.25 / (kap * d0);')],
    'sub8': [('tpe_device.h', 'constexpr int kBxSubBits = 4;', 'constexpr int kBxSubBits = 3;')],
    'fin32': [('tpe_engine.hip', 'hipLaunchKernelGGL(k_rescore_fin, dim3((unsigned)std::min<int64_t>(ne_sliced, 256))',
               'hipLaunchKernelGGL(k_rescore_fin, dim3((unsigned)std::min<int64_t>(ne_sliced, 32))')],
    'mt16': [('tpe_engine.hip', 'constexpr int64_t kHotMinTiles = 6;', 'constexpr int64_t kHotMinTiles = 16;')],
    'bm': [('tpe_device.h',
            '    return __builtin_amdgcn_sqrt(fmax(0.0, 2.0 * bm_neglog(u01_open0(y), lt)));\n',
            '    return (double)y * 0x1.0p-31;\n')],
    'lb4': [('tpe_engine.hip', '__launch_bounds__(kBlock, 6) void k_hot_bx(',
             '__launch_bounds__(kBlock, 4) void k_hot_bx(')],
    'lb5': [('tpe_engine.hip', '__launch_bounds__(kBlock, 6) void k_hot_bx(',
             '__launch_bounds__(kBlock, 5) void k_hot_bx(')],
    'bxlb4': [('tpe_expand.hip', '__global__ __launch_bounds__(kBlock) void k_bx_table(',
               '__global__ __launch_bounds__(kBlock, 4) void k_bx_table(')],
    'nopieces': [('tpe_engine.hip', 'res_bytes >= ((size_t)8 << 20)', 'res_bytes >= ((size_t)1 << 62)')],
    'bx3': [('tpe_expand.hip', 'constexpr int kBxChains = 4;', 'constexpr int kBxChains = 3;')],
    'bx2': [('tpe_expand.hip', 'constexpr int kBxChains = 4;', 'constexpr int kBxChains = 2;')],
    'nolist': [('tpe_engine.hip', '            const uint64_t bal = __ballot(take);\n            if (!bal) continue;\n            const int c = __builtin_amdgcn_readfirstlane',
                '            const uint64_t bal = __ballot(take && (pend >> 31));\n            if (!bal) continue;\n            const int c = __builtin_amdgcn_readfirstlane')],
    'nolist2': [('tpe_engine.hip', '            const uint64_t bal = __ballot(take);\n            if (!bal) continue;\n            const int c = __builtin_amdgcn_readfirstlane',
                 '            const uint64_t bal = __ballot(x[r] == 1234.5678);\n            if (!bal) continue;\n            const int c = __builtin_amdgcn_readfirstlane')],
    'norej': [('tpe_device.h',
               '    const bool bounded = (L.flags & 3) == 3;\n    const uint32_t mask0 = pend;',
               '    const bool bounded = false;\n    const uint32_t mask0 = pend;')],
}


def main(name, defs):
    tmp = tempfile.mkdtemp(prefix='tpe_variant_')
    try:
        csrc = os.path.join(tmp, 'hyperopt_amd', 'csrc')   # (the sources include ../../include/)
        rev = os.environ.get('VARIANT_REV')   # the sources of another commit (timing comparisons)
        if rev:
            import subprocess
            for sub in ('hyperopt_amd/csrc', 'include'):
                out = subprocess.check_output(['git', '-C', REPO, 'archive', rev, sub])
                subprocess.run(['tar', '-x', '-C', tmp], input=out, check=True)
        else:
            shutil.copytree(os.path.join(REPO, 'hyperopt_amd', 'csrc'), csrc)
            shutil.copytree(os.path.join(REPO, 'include'), os.path.join(tmp, 'include'))
        for fname, old, new in PATCHES.get(name, []):
            p = os.path.join(csrc, fname)
            txt = open(p).read()
            if old not in txt:
                raise SystemExit('patch %s does not apply to %s' % (name, fname))
            open(p, 'w').write(txt.replace(old, new, 1))
        srcs = [os.path.join(csrc, os.path.basename(s)) for s in _build.SOURCES]
        deps = [os.path.join(csrc, os.path.basename(d)) if '/csrc/' in d else d for d in _build.DEPS]
        h = hashlib.sha256((_build.source_hash(deps) + ' '.join(defs)).encode()).hexdigest()
        stamp = ('v:%s:%s' % (name, h))[:16]
        _build.SOURCES = srcs
        _build.source_hash = lambda deps=None: stamp
        _build.FLAGS = _build.FLAGS + list(defs)
        _build.TARGET = os.path.join(HERE, 'var_%s.so' % name)
        _build.build_engine(force=True, verbose=False)
        print('built %s (stamp %s)' % (_build.TARGET, stamp))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2:])

#!/bin/bash
# One gpurun call: the named steps in order, each under its own time limit,
# output under gpurun_out/<tag>/; the call stops at the first failing step.
#
#   bash tools/gpu.sh <tag> <step> [<step> ...]
#
# steps:
#   tests            the whole -m gpu suite (one pytest process)
#   tests=<expr>     the -m gpu tests matching pytest -k <expr> (commas for spaces)
#   smoke            __graft_entry__.smoke()
#   bench            the default bench.py line (what the driver runs)
#   bench=<args>     bench.py with extra arguments (commas for spaces)
#   var=<name>[,args] bench.py on the variant library tools/var_<name>.so (tools/build_variant.py)
#   htrace=<script,args> rocprofv3 kernel + memory-copy + HIP API trace of a script -> <tag>/htrace<n>
#   vpy=<name>,<script,args> a python script of the tree on that variant library
#   trace=<args>     rocprofv3 --kernel-trace --stats of bench.py <args> -> <tag>/trace<n>
#   prof             tools/prof_round.sh <tag> (kernel trace + PMC passes of the default line)
#   lpdf             the plain fp64 round's trace + PMC passes (tools/prof_round.sh <tag>_lpdf)
#   shard=<r>        label shard r of config 3 alone: probe + kernel/HIP-API trace
#   py=<script,args> any python script of the tree (commas for spaces)
#   ubench           tools/ubench_issue (built beforehand): VALU issue costs -> issue_costs.json
#   listpmc          rocprofv3 --list-avail (the counters this box offers)
#   bm32             tools/ubench_bm32 (built beforehand): exhaustive fp32 Box-Muller error sweep
#   ab               tools/ab_hot.py (option A/B in one process), its trace and PMC passes -> profiles/<tag>_ab_*
set -u
T=${1:?tag}
shift
OUT=gpurun_out/$T
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"

run() {   # run <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    echo "== $name: $*"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -n 4 "$OUT/$name.log"
    echo "== $name rc=$rc"
    return $rc
}

n=0
for s in "$@"; do
    n=$((n + 1))
    case "$s" in
        tests)   # (a failed test -- pytest rc 1 -- does not stop the later steps; anything else does)
            run tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
            rc=$?; [ $rc -le 1 ] || exit 1 ;;
        tests=*)
            k=${s#tests=}
            run tests$n 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "${k//,/ }"
            rc=$?; [ $rc -le 1 ] || exit 1 ;;
        smoke)
            run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
        bench)
            run bench 600 python -u bench.py || exit 1 ;;
        bench=*)
            a=${s#bench=}
            run bench$n 600 python -u bench.py ${a//,/ } || exit 1 ;;
        vtests=*)   # -m gpu tests on a variant library: vtests=<name>,<pytest -k expr, commas for spaces>
            a=${s#vtests=}
            v=${a%%,*}
            k=${a#*,}
            run vtests_$v$n 600 env HYPEROPT_AMD_VARIANT=tools/var_$v.so python -u -m pytest tests -m gpu -v \
                --timeout 300 --timeout-method thread -k "${k//,/ }"
            rc=$?; [ $rc -le 1 ] || exit 1 ;;
        var=*)   # bench.py on a tools/build_variant.py library: var=<name>[,bench args]
            a=${s#var=}
            v=${a%%,*}
            rest=""; [ "$a" != "$v" ] && rest=${a#*,}
            run var_$v$n 600 env HYPEROPT_AMD_VARIANT=tools/var_$v.so python -u bench.py ${rest//,/ } || exit 1 ;;
        vpy=*)   # a python script of the tree on a variant library: vpy=<name>,<script>[,args]
            a=${s#vpy=}
            v=${a%%,*}
            rest=${a#*,}
            run vpy_$v$n 600 env HYPEROPT_AMD_VARIANT=tools/var_$v.so python -u ${rest//,/ } || exit 1 ;;
        htrace=*)   # kernel + copy + HIP API trace of a python script: htrace=<script,args>
            a=${s#htrace=}
            run htrace$n 400 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d "$OUT/htrace$n" -o run \
                --output-format csv -- python -u ${a//,/ } || exit 1 ;;
        trace=*)   # rocprofv3 kernel trace + stats of bench.py with these arguments (commas for spaces)
            a=${s#trace=}
            run trace$n 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace$n" -o run --output-format csv \
                -- python -u bench.py ${a//,/ } || exit 1 ;;
        prof)
            bash tools/prof_round.sh "$T" --steps 5 --warmup 2 --no-other-configs --no-agreement || exit 1 ;;
        lpdf)   # the plain fp64 round (k_round<double>, no screen) at config 3: trace + PMC passes
            bash tools/prof_round.sh "${T}_lpdf" --mode warm --no-screen --steps 2 --warmup 1 || exit 1 ;;
        shard=*)
            r=${s#shard=}
            run shard$r 200 python -u tools/shard_probe.py "$r" 20 || exit 1
            run shard${r}_trace 240 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --stats \
                -d "$OUT/shard${r}_trace" -o run --output-format csv -- python -u tools/shard_probe.py "$r" 10 || exit 1 ;;
        ubench)
            echo "== ubench"
            timeout -k 10 120 tools/ubench_issue > "$OUT/issue_costs.json" 2> "$OUT/ubench.err" || { cat "$OUT/ubench.err"; exit 1; }
            cat "$OUT/issue_costs.json" ;;
        bm32)
            run bm32 300 tools/ubench_bm32 || exit 1
            grep -q "BOUNDS HOLD" "$OUT/bm32.log" || { echo "fp32 Box-Muller bounds violated"; exit 1; } ;;
        absplit)   # tools/ab_hot.py over index window splits 1, 2, 4, 8 (the hot32 A/B too)
            run absplit 300 env AB_SPLITS=1,2,4,8 python -u tools/ab_hot.py 6 || exit 1 ;;
        ab)      # tools/ab_hot.py: hot32 0/1 and bx_split 1/auto alternating, its kernel trace and PMC passes
            run ab 300 python -u tools/ab_hot.py 8 || exit 1
            run ab_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
                -- python -u tools/ab_hot.py 2 || exit 1
            for p in "valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                     "mix SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE" \
                     "mix32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
                     "stall SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"; do
                set -- $p
                name=$1; shift
                echo "== pmc_$name"
                timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$OUT/pmc_$name" -o run --output-format csv \
                    -- python -u tools/ab_hot.py 1 > "$OUT/pmc_$name.log" 2>&1 || { tail -5 "$OUT/pmc_$name.log"; exit 1; }
            done
            python tools/pmc_summary.py "$OUT" "${T}_ab" > /dev/null || exit 1 ;;
        listpmc)
            run listpmc 120 rocprofv3 --list-avail || exit 1 ;;
        py=*)
            a=${s#py=}
            run py$n 600 python -u ${a//,/ } || exit 1 ;;
        *)
            echo "unknown step $s"; exit 2 ;;
    esac
done
echo "== all steps done"

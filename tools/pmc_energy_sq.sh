set -o pipefail
R=$(pwd); O=$R/gpurun_out/pmc_r2i; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $O -o p1 -- python $R/bench.py --config energy --steps 1 --warmup 0 --batch 64 --no-cpu-baseline > $O/p1.log 2>&1 || exit 1
echo done

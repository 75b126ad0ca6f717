set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pp
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/photo_one.py 12 12 > $R/gpurun_out/pp/plain.txt 2>&1
rocprofv3 -L > /tmp/counters.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" /tmp/counters.txt | sort -u > $R/gpurun_out/pp/sq_counters.txt || true
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/pp/p1 -o run --output-format csv -- python3 $R/tools/photo_one.py 12 4 > /dev/null 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $R/gpurun_out/pp/p2 -o run --output-format csv -- python3 $R/tools/photo_one.py 12 4 > /dev/null 2>&1
echo done

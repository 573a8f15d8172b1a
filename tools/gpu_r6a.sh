set -o pipefail
R=$(pwd); O=$R/gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/resident_sweep.py --ntraj 256 1x1024 1x64 1x16 1x8 1x4 2x8 2x4 4x4 4x2 4x1 > $O/r6a_resident.txt 2>&1 || { tail -20 $O/r6a_resident.txt; exit 1; }
cat $O/r6a_resident.txt
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r6a_b8 -o kt -- python $R/tools/resident_sweep.py --ntraj 64 1x8 4x2 > $O/prof_r6a_b8.log 2>&1 || { tail -20 $O/prof_r6a_b8.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_r6a_b8 -o fetch -- python $R/tools/resident_sweep.py --ntraj 16 1x8 > $O/pmc_r6a_b8_f.log 2>&1 || { tail -20 $O/pmc_r6a_b8_f.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_r6a_b8 -o write -- python $R/tools/resident_sweep.py --ntraj 16 1x8 > $O/pmc_r6a_b8_w.log 2>&1 || { tail -20 $O/pmc_r6a_b8_w.log; exit 1; }
echo r6a done

set -u
mkdir -p gpurun_out
BNFLAC_PW_STATS=1 timeout -k 10 200 python tools/pw_stats.py C2 1 > gpurun_out/r3p_pw.log 2>&1 || { tail gpurun_out/r3p_pw.log; exit 1; }
cat gpurun_out/r3p_pw.log
BNFLAC_PW_STATS=1 timeout -k 10 200 python tools/pw_stats.py C5 1 >> gpurun_out/r3p_pw.log 2>&1 || { tail gpurun_out/r3p_pw.log; exit 1; }
tail -5 gpurun_out/r3p_pw.log

export TMPDIR=/tmp
for cfg in "X=0" "WHISPER_MI355X_BDEC_SKIP=3"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python -u tools/bdec_stamps.py large-v3+conf BF16 128 24 > gpurun_out/r05l_exp.txt 2>&1 || { echo FAIL; tail -5 gpurun_out/r05l_exp.txt; exit 1; }
  grep -E "T2|T4|T5|H1 |H3|H5|span" gpurun_out/r05l_exp.txt
done

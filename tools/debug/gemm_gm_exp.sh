# encoder tile order A/B: phases.encode.ms of the headline bench per WHISPER_MI355X_GEMM_GM
export TMPDIR=/tmp
for gm in 0 4 8 16; do
  WHISPER_MI355X_GEMM_GM=$gm timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --variants 0 --app-pattern 0 --cpu-baseline 0 --frontend 0 --f16-line 0 > gpurun_out/r05l_gm$gm.txt 2>&1 || { echo "gm=$gm FAIL"; tail -3 gpurun_out/r05l_gm$gm.txt; exit 1; }
  echo "gm=$gm $(grep -o '"value": [0-9.]*' gpurun_out/r05l_gm$gm.txt | head -1) $(grep -o '"encode": {"bound": "mfma", "ms": [0-9.]*' gpurun_out/r05l_gm$gm.txt | head -1)"
done

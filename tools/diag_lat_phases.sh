cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
for v in stamps noz nogemm stamps; do
 timeout -k 10 60 python tools/trace_lat.py build/libmfgp_$v.so > gpurun_out/diag_$v.txt 2>&1 || { tail -5 gpurun_out/diag_$v.txt; exit 1; }
 echo "== $v"; grep -E "last WG end|w unit    slot 2|Z unit    slot 2|gemm      slot (1|2|4)" gpurun_out/diag_$v.txt
done

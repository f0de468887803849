cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
for wu in 512 256 128; do for ks in 8 4 2; do
 echo "== WU=$wu KS=$ks"; TRACE_B=1 MFGP_LAT_WU=$wu MFGP_LAT_KSPLIT=$ks timeout -k 10 60 python tools/trace_lat.py build/libmfgp_stamps.so > gpurun_out/sw_${wu}_${ks}.txt 2>&1 || exit 1
 grep -E "last WG end|F loop|reduce\+L22|K-loop dur" gpurun_out/sw_${wu}_${ks}.txt
done; done

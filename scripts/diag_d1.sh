mkdir -p gpurun_out/d1
for v in prof notf8; do echo "== $v"; WISER_HIP_LIB=$PWD/wiser_amd/_lib/var_$v/libwiser_hip.so timeout -k 10 300 python3 scripts/diag_types.py --only high-high || exit 1; done

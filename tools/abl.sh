# conv ablation timings: the HN_EXPERIMENTS library (make -C hardnetnas_amd/csrc abl) holds the
# timing-only builds; the product library rejects them.
export HN_LIB=abl/libhardnet_mi355x.so
python tools/tune_variants.py "001000" > gpurun_out/abl0.log 2>&1 && HN_DEBUG=1 python tools/tune_variants.py "001000" > gpurun_out/abl1.log 2>&1; tail -1 gpurun_out/abl0.log; tail -1 gpurun_out/abl1.log

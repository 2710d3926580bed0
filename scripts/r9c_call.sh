# round-6 GPU bundle 24: config-4 stem int8 epilogue as med3 + v_cvt_pk_u8 (relu) -- stem and
# int8 model tests, config-4 step trace and benches
bash scripts/gpu.sh r9c "tests:stem or int8 or i8" profc4 cfg4

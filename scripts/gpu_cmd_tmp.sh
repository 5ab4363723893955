bash scripts/gpu_ab_env.sh g8ab3 PG_FP8_GEMV "1 0" 2 --config pt-896 --batch 32 --fp8 --steps 2 --warmup 1

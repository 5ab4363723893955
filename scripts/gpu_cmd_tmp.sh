bash scripts/gpu_suite.sh r4a && bash scripts/gpu_profile.sh r4ap long

for d in /sys/class/drm/card*/device; do echo "== $d"; ls $d | tr '\n' ' ' | head -c 2500; echo; cat $d/pp_dpm_sclk 2>&1 | head -20; cat $d/current_link_speed 2>&1 | head -2; ls -la $d/gpu_metrics 2>&1; done
which amd-smi rocm-smi; amd-smi version 2>&1 | head -3

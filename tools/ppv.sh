mkdir -p gpurun_out
for n in BASE DMAC NODMA NOREAD NONE; do
  CLM_LIB=tools/libclm_$n.so timeout -k 10 120 python -u tools/pp_probe.py 12 v_fc1,t_fc1,v_qkv > gpurun_out/ppv_$n.jsonl 2>&1 || exit 1
done

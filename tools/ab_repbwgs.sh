# rep backward workgroup count (VAESNE_REP field 6: 1536 default) after the summed-dO rewrite:
# fewer (512: a free wave slot per SIMD for the encoder chain beside it) or more, shorter
# workgroups (3072 / 6144: slots recycle faster)
bash profiles/ab_env.sh "VAESNE_REP=0,2,256,1,16,1536,1" "VAESNE_REP=0,2,256,1,16,512,1" \
  "VAESNE_REP=0,2,256,1,16,3072,1" "VAESNE_REP=0,2,256,1,16,6144,1" > gpurun_out/ab_bwgs.txt 2>&1

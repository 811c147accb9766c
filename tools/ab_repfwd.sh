# A/B of the block-1 (repeated-sequence) attention forward geometry: copies per
# workgroup (frc) and threads (fnt).  RC=4 runs at 159 VGPRs / half the waves, leaving
# room beside it for the spectra encoder's chain of small kernels.
bash profiles/ab_env_list.sh "VAESNE_REP=0,2,256,1,16,1536,1" "VAESNE_REP=0,4,256,1,16,1536,1" \
  "VAESNE_REP=128,4,256,1,16,1536,1" "VAESNE_REP=0,2,256,1,16,1536,2"

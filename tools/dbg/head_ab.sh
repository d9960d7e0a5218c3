O=gpurun_out; : > $O/r05w_head_ab.txt
for r in 1 2 3; do for L in hilp0 . hf8 hf16; do
  echo "== $L round $r" >> $O/r05w_head_ab.txt
  EBC_LIB_PATH=$PWD/clip-ebc_amd/lib/$L/libebc_hip.so timeout -k 10 120 python -u tools/kbench.py head 16 --reps 200 >> $O/r05w_head_ab.txt 2>&1 || exit 1
done; done

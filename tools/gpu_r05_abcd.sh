export LD_LIBRARY_PATH=ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/otfuse/lib
mkdir -p gpurun_out/cd
for r in 1 2; do for b in st_pw st_pwA st_pwD; do
  timeout -k 10 120 ./tools/$b 4096 100 pw > gpurun_out/cd/$b.$r.txt 2>&1 || exit 1
  echo "$b $r $(grep solve gpurun_out/cd/$b.$r.txt | tail -3 | awk '{print $5}' | tr '\n' ' ') status $(grep -c 'status=2' gpurun_out/cd/$b.$r.txt) loop $(grep 'K formed -> loop' gpurun_out/cd/$b.$r.txt)"
done; done

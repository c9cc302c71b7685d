# stress the epilogues of several builds: base (the in-tree _C), and exp/variants/_C_<name>.so
rm -f gpurun_out/variants.log
for v in base ${VARIANTS}; do
  if [ $v = base ]; then unset FLUXMPI_C_VARIANT; else export FLUXMPI_C_VARIANT=exp/variants/_C_$v.so; fi
  echo "== $v" >> gpurun_out/variants.log
  timeout -k 10 150 python scripts/diag/epi_stress.py >> gpurun_out/variants.log 2>&1 || exit 1
done

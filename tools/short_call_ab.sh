set -e
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 60 ./build/short_call_timer 2000 > gpurun_out/r06m_sct_new_$i.json
  timeout -k 10 60 ./build/short_call_timer_ref 2000 > gpurun_out/r06m_sct_ref_$i.json
done
CASES=gsdrFirFC,gsdrFmDemod,gsdrAmDemod,gsdrxFirFCInt8,gsdrxFmDemodInt8 timeout -k 10 400 python -u tools/ab_ref.py build/ref_23c4540/libgsdr.so > gpurun_out/r06m_ab.txt 2>&1

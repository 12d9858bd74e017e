cd ${GRAFT_REPO_ROOT} && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fwdmodes -o m -- python3 scripts/m256_fwd_modes.py > gpurun_out/fwdmodes.log 2>&1 && python3 -c "
import csv
rows=[r for r in csv.DictReader(open('gpurun_out/fwdmodes/m_kernel_trace.csv')) if 'k_dec256_fwd' in r['Kernel_Name']]
rows.sort(key=lambda r:int(r['Start_Timestamp']))
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows]
print('train', [round(x) for x in d[0:4]+d[8:12]]); print('infer', [round(x) for x in d[4:8]+d[12:16]])"

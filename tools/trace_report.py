import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
idx=[i for i,r in enumerate(rows) if 'wf_generate' in r['Kernel_Name'] or 'megakernel' in r['Kernel_Name']]
last=rows[idx[-1]:]
tot=0
for r in last:
    d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3; tot+=d
    name=r['Kernel_Name'].split('(')[0].replace('void ','')
    if 'rocclr' in name: continue
    print(f"{name:34s} {d:9.1f} us grid {int(r['Grid_Size_X'])//256:6d} blk vgpr {r['VGPR_Count']} lds {r['LDS_Block_Size']}")
print('sum', tot)

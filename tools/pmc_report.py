import csv, collections, glob, sys
agg=collections.defaultdict(lambda: collections.defaultdict(float))
d = sys.argv[2] if len(sys.argv) > 2 else 'gpurun_out/pmc'
for f in sorted(glob.glob(d + '/p*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        k=r['Kernel_Name'].split('(')[0].replace('void ','')
        if 'rocclr' in k: continue
        agg[k][r['Counter_Name']]+=float(r['Counter_Value'])
flt = sys.argv[1] if len(sys.argv)>1 else ''
for k,v in agg.items():
    if flt not in k: continue
    print(k)
    for c,x in sorted(v.items()): print('   %-34s %.4g'%(c,x))
    g=lambda n: v.get(n,0)
    if g('SQ_WAVE_CYCLES'):
        print('   -> wait_any %.2f wait_inst %.2f valu %.2f'%(g('SQ_WAIT_ANY')/g('SQ_WAVE_CYCLES'), g('SQ_WAIT_INST_ANY')/g('SQ_WAVE_CYCLES'), g('SQ_ACTIVE_INST_VALU')/g('SQ_WAVE_CYCLES')))
    if g('SQ_ACTIVE_INST_VALU') and g('SQ_THREAD_CYCLES_VALU'): print('   -> lane util %.3f'%(g('SQ_THREAD_CYCLES_VALU')/(64*g('SQ_ACTIVE_INST_VALU'))))
    if g('TCP_TCC_READ_REQ_sum'): print('   -> avg L2 read latency %.1f cyc'%(g('TCP_TCC_READ_REQ_LATENCY_sum')/g('TCP_TCC_READ_REQ_sum')))
    # occupancy: SQ_WAVE_CYCLES counts quad-cycles summed over every wave; GRBM_GUI_ACTIVE is summed
    # over the 8 XCDs (MI355X_MICROARCH.md), so the launch lasted GRBM_GUI_ACTIVE / 8 cycles on 1,024
    # SIMDs (SQ_LEVEL_WAVES reads 0 on gfx950: the old line printed 0.0 every round)
    if g('GRBM_GUI_ACTIVE') and g('SQ_WAVE_CYCLES'):
        print('   -> avg waves resident per SIMD %.2f'%(4*g('SQ_WAVE_CYCLES')/(g('GRBM_GUI_ACTIVE')/8)/1024))
    if g('GRBM_GUI_ACTIVE') and g('SQ_INSTS_VALU'):
        print('   -> VALU issue fraction %.3f (2 cycles per wave-instruction, 1,024 SIMDs)'%(2*g('SQ_INSTS_VALU')/(1024*g('GRBM_GUI_ACTIVE')/8)))
    if g('SQ_INSTS_VMEM_RD') and g('SQ_INST_LEVEL_VMEM'): print('   -> avg VMEM instr latency %.0f cyc (level / instrs)'%(g('SQ_INST_LEVEL_VMEM')/(g('SQ_INSTS_VMEM_RD')+g('SQ_INSTS_VMEM_WR'))))

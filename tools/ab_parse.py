import csv,glob,sys
for tag in sys.argv[1:]:
    for run in ('base_1','prev_1','base_2','prev_2'):
        fs=glob.glob('gpurun_out/%s/%s/*kernel_stats.csv'%(tag,run))
        if not fs: continue
        out=[]
        for r in csv.DictReader(open(fs[0])):
            n=r['Name']
            if 'key_fast' in n or 'key_asm' in n or 'bgzf_wave' in n or 'scan_mfma' in n:
                sh='big' if 'KfShapeILi1024' in n or '<1024' in n else ('small' if 'key_fast' in n else n[:30].split('(')[0])
                out.append('%s calls=%s avg=%.1fus'%(sh,r['Calls'],float(r['AverageNs'])/1e3))
        print(tag,run,' | '.join(out))

"""Phase timeline of the last warm fit in a rocprofv3 kernel trace (tools/fit_timing.py under
--kernel-trace):  python tools/fit_timeline.py <rocprof output dir>"""
import csv,sys
d=sys.argv[1]
rows=list(csv.DictReader(open(f'{d}/run_kernel_trace.csv')))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
fills=[i for i,r in enumerate(rows) if 'rbf_fill' in r['Kernel_Name']]
i=fills[-1]
j=max(k for k,r in enumerate(rows) if 'tile_box' in r['Kernel_Name'])
start=int(rows[i]['Start_Timestamp'])
def ms(x): return (int(x)-start)/1e6
print(d,'fill->tile_box end %.1f'%ms(rows[j]['End_Timestamp']))
marks={}
for r in rows[i:j+1]:
    n=r['Kernel_Name']
    for key in ['chol_diag','chol_trsm','syrk','SB_MT','widen_kernel','trtri','DB_MT','widen_sub','pack_operand','row_l1','tile_norm','tile_box','predict']:
        if key in n:
            m=marks.setdefault(key,[1e9,0,0,0]); m[0]=min(m[0],ms(r['Start_Timestamp'])); m[1]=max(m[1],ms(r['End_Timestamp'])); m[2]+=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6; m[3]+=1
for k,v in sorted(marks.items(),key=lambda x:x[1][0]): print('%-14s [%.1f, %.1f] busy %.1f n=%d'%(k,*v))
dg=[r for r in rows[i:j+1] if 'chol_diag' in r['Kernel_Name']]
st=[ms(r['Start_Timestamp']) for r in dg]
print('diag starts every 16:', ' '.join('%.1f'%x for x in st[::16]), 'last end %.1f'%ms(dg[-1]['End_Timestamp']))
print('diag dur avg first/second half: %.1f %.1f us'%(sum(int(r['End_Timestamp'])-int(r['Start_Timestamp']) for r in dg[:64])/64e3, sum(int(r['End_Timestamp'])-int(r['Start_Timestamp']) for r in dg[64:])/len(dg[64:])/1e3))
tr=[r for r in rows[i:j+1] if 'chol_trsm' in r['Kernel_Name']]
print('trsm dur avg first/second half: %.1f %.1f us'%(sum(int(r['End_Timestamp'])-int(r['Start_Timestamp']) for r in tr[:64])/64e3, sum(int(r['End_Timestamp'])-int(r['Start_Timestamp']) for r in tr[64:])/len(tr[64:])/1e3))

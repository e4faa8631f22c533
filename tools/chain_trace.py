import csv,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
# take last build: find last k_pack_line
idx=[i for i,r in enumerate(rows) if 'k_pack_line' in r['Kernel_Name']]
st=idx[-1]
t0=int(rows[st]['Start_Timestamp'])
n=0
for r in rows[st:st+int(sys.argv[2])]:
    nm=r['Kernel_Name'].split('(')[0].replace('void ','')[:40]
    s=(int(r['Start_Timestamp'])-t0)/1e3; e=(int(r['End_Timestamp'])-t0)/1e3
    print(f"{nm:40s} q{r.get('Queue_Id','?'):>3} grid{r['Grid_Size_X']:>7}x{r['Grid_Size_Y']} {s:9.1f} {e:9.1f} {e-s:7.1f}")

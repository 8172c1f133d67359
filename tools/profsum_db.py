import sqlite3, sys
db=sqlite3.connect(sys.argv[1])
cur=db.cursor()
q='''select s.kernel_name, count(*), sum(d.end-d.start)/1e6, avg(d.end-d.start)/1e3 from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id=s.id group by s.kernel_name order by 3 desc'''
rows=list(cur.execute(q)); tot=sum(r[2] for r in rows)
n=int(sys.argv[2]) if len(sys.argv)>2 else 25
for r in rows[:n]: print("%-62s %8d %10.1f ms %8.2f us %5.1f%%"%(r[0][:62],r[1],r[2],r[3],100*r[2]/tot))
print('total kernel ms %.1f  span s %s'%(tot, [ (b-a)/1e9 for a,b in cur.execute('select min(start), max(end) from rocpd_kernel_dispatch')]))

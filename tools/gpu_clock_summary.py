"""Per-slot GPU-clock stages of a GSS_RUN_TRACE=1 gss_run log ("trace gpu" lines, HIP events
on the run's streams): upload (start -> kernels), render kernels (-> rendered), the download
(copy start -> done), how long a rendered slot waited for the copy engine, and the interval
between downloads finished, medians over the last run in the log.

usage: python tools/gpu_clock_summary.py <stderr log>"""
import sys, statistics as S
L=[l for l in open(sys.argv[1]) if l.startswith('trace gpu')]
runs=[];cur=[]
for l in L:
    f=l.split(); first=int(f[3]); a,k,b,c,q=float(f[5]),float(f[7]),float(f[9]),float(f[11]),float(f[13])
    if cur and first < cur[-1][0]: runs.append(cur); cur=[]
    cur.append((first,a,k,b,c,q))
runs.append(cur)
r=runs[-1]
print("slots",len(r),"median h2d %.3f kern %.3f d2h(done-copy) %.3f copy_wait(copy-rendered) %.3f interval %.3f"%(S.median(x[2]-x[1] for x in r),S.median(x[3]-x[2] for x in r),S.median(x[4]-x[5] for x in r),S.median(x[5]-x[3] for x in r),S.median(r[i][4]-r[i-1][4] for i in range(1,len(r)))))

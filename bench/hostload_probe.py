import time
def snap():
    d={}
    for l in open('/proc/stat'):
        if l.startswith('cpu') and l[3].isdigit():
            f=l.split(); c=int(f[0][3:]); v=list(map(int,f[1:]))
            idle=v[3]+v[4]; d[c]=(sum(v),idle)
    return d
a=snap(); time.sleep(2); b=snap()
busy={c:1-(b[c][1]-a[c][1])/max(1,(b[c][0]-a[c][0])) for c in a}
tot=sum(busy.values())
print("total busy cpus: %.1f"%tot)
print("busiest:", sorted(((round(v,2),c) for c,v in busy.items()), reverse=True)[:40])
import os
for c in (0,8,64,128):
    p=f"/sys/devices/system/cpu/cpu{c}/cache/index3/id"
    print(c, open(p).read().strip() if os.path.exists(p) else None, open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip())

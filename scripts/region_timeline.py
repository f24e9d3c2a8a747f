"""Split the regions of scripts/region_trace.py (rocprofv3 --kernel-trace --hip-runtime-trace, csv)
into hipGraphLaunch -> first kernel start, the K kernels, and last kernel end -> synchronize
return.  argv[1] = the rocprofv3 output directory.  Profiler overhead inflates the host side."""
import csv,sys
d=sys.argv[1]
api=list(csv.DictReader(open(d+"/run_hip_api_trace.csv")))
ker=list(csv.DictReader(open(d+"/run_kernel_trace.csv")))
ker=[k for k in ker if "step_kernel" in k["Kernel_Name"]]
ker.sort(key=lambda k:int(k["Start_Timestamp"]))
launch=[a for a in api if a["Function"]=="hipGraphLaunch"]
syncs=[a for a in api if "Synchronize" in a["Function"]]
print(len(launch),len(ker),set(a["Function"] for a in api if int(a["Start_Timestamp"])>int(launch[0]["Start_Timestamp"])))
for L in launch[1:]:
    ls,le=int(L["Start_Timestamp"]),int(L["End_Timestamp"])
    ks=[k for k in ker if int(k["Start_Timestamp"])>=ls][:20]
    if len(ks)<20: continue
    s=[a for a in syncs if int(a["Start_Timestamp"])>=le][0]
    k0=int(ks[0]["Start_Timestamp"]); kN=int(ks[-1]["End_Timestamp"])
    durs=[(int(k["End_Timestamp"])-int(k["Start_Timestamp"]))/1e3 for k in ks]
    gaps=[(int(ks[i+1]["Start_Timestamp"])-int(ks[i]["End_Timestamp"]))/1e3 for i in range(19)]
    print(f"launch api {(le-ls)/1e3:6.1f}  launch->k0 {(k0-ls)/1e3:6.1f}  kernels {(kN-k0)/1e3:6.1f} (k0 {durs[0]:.2f} k1 {durs[1]:.2f} mean {sum(durs)/20:.2f} gapmean {sum(gaps)/19:.2f})  kN->sync end {(int(s['End_Timestamp'])-kN)/1e3:6.1f}  total {(int(s['End_Timestamp'])-ls)/1e3:6.1f} sync-fn {s['Function']}")

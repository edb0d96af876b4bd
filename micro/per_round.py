"""Per-round durations of a kernel from a rocprofv3 kernel trace: launches in time order, index modulo 10
(the mapping rounds of a frame), median / max per round after the first 10 frames. Profiling aid only.

usage: python micro/per_round.py gpurun_out/NAME/run_kernel_trace.csv k_map_assoc [k_lm_coop ...]"""
import csv,collections,sys
r=list(csv.DictReader(open(sys.argv[1])))
for name in sys.argv[2:]:
    a=[x for x in r if name in x['Kernel_Name']]
    a.sort(key=lambda x:int(x['Start_Timestamp']))
    d=collections.defaultdict(list)
    for i,x in enumerate(a): d[i%10].append((int(x['End_Timestamp'])-int(x['Start_Timestamp']))/1e3)
    print(name, ' '.join('%d:%.1f/%.1f'%(k, sorted(d[k][10:])[len(d[k][10:])//2], max(d[k][10:])) for k in sorted(d)))

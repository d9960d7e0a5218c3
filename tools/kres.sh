#!/bin/bash
# Per-kernel resource usage (VGPR/AGPR/SGPR/spills/LDS) of a built object: tools/kres.sh clip-ebc_amd/build/gemm.o [regex]
set -e
o=$(readlink -f $1); f=${2:-.}
tmp=$(mktemp -d); cd $tmp; cp $o k.o
/opt/rocm/lib/llvm/bin/llvm-objdump --offloading k.o > /dev/null
co=$(ls k.o.*gfx950* | head -1)
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $co | grep -E "\.name:|vgpr_count|agpr_count|sgpr_count|spill_count|group_segment_fixed_size|private_segment_fixed_size" | \
python3 -c "
import sys,re
recs=[];cur=None
for l in sys.stdin:
    l=l.strip()
    k,_,v=l.partition(':'); k=k.strip().lstrip('.').lstrip('- ').lstrip('.'); v=v.strip()
    if k=='name':
        if cur: recs.append(cur)
        cur={'name':v}
    elif cur is not None: cur[k]=v
if cur: recs.append(cur)
for r in recs:
    if re.search(sys.argv[1], r.get('name','')):
        print('v',r.get('vgpr_count'),'a',r.get('agpr_count'),'s',r.get('sgpr_count'),'spill',r.get('vgpr_spill_count'),r.get('sgpr_spill_count'),'lds',r.get('group_segment_fixed_size'),'priv',r.get('private_segment_fixed_size'),r['name'][:110])
" "$f"
cd /; rm -rf $tmp

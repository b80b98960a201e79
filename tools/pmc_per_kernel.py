"""Per-kernel VALU count, busy cycles and issue utilisation from rocprofv3
PMC passes (tools/gpu/pmc_lib.sh: SQ_INSTS_VALU, GRBM_GUI_ACTIVE, SQ_WAVES;
dispatches serialise under --pmc, so each kernel is measured alone).
    python tools/pmc_per_kernel.py gpurun_out/pmc_<a> [gpurun_out/pmc_<b> ...]
util = VALU x 4 cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)."""
import csv,sys,glob,re,collections
for d in sys.argv[1:]:
    f=glob.glob(d+'/**/*counter_collection.csv',recursive=True)[0]
    acc=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.Counter()
    for r in csv.DictReader(open(f)):
        k=re.sub(r'\(.*','',r['Kernel_Name'].replace('noise_amd::','').replace('void ',''))
        acc[k][r['Counter_Name']]+=float(r['Counter_Value'])
        if r['Counter_Name']=='SQ_INSTS_VALU': n[k]+=1
    print('==',d)
    tv=0;tc=0
    for k in sorted(acc):
        if not any(x in k for x in ('tile', 'seg', 'cls', 'unit')): continue
        v=acc[k]['SQ_INSTS_VALU']/n[k]; g=acc[k]['GRBM_GUI_ACTIVE']/n[k]/8
        print('%-50s valu %8.1fM cyc %8.0fk util %.3f'%(k[:50],v/1e6,g/1e3,v*4/1024/g if g else 0))

for rep in 1 2; do for ov in ${OVS:-1 0}; do for w in ${WS:-C3 C5}; do
TFBS_PREP_OVERLAP=$ov timeout -k 10 400 python3 bench.py --workload $w --no-cpu > gpurun_out/pab_${w}_${ov}_$rep.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/pab_${w}_${ov}_$rep.json'));e=d['end_to_end'];print('$w ov=$ov rep$rep', round(e['regions_per_s']), {k:round(v,3) for k,v in e['rank0_phases_s'].items() if k in ('host_prep_wall','build_region_thread_s','rows_bgzf')})"
done; done; done

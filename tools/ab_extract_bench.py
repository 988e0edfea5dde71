"""Summarise tools/ab.sh lines of full bench.py runs (AB_CMD="bench.py --no-cpu-baseline"): headline, config 4, steady iteration, IL steps."""
import json,sys
for line in sys.stdin:
    v, _, js = line.partition(' ')
    try: j=json.loads(js)
    except Exception: continue
    s=j['secondary']
    print(v, round(j['value']/1e9,4), 'c4box100', round(s['config4_cartpole_box100']['value']/1e9,4), 'c4box10', round(s['config4_cartpole_box10']['value']/1e9,4), 'steady', round(j['roofline_steady_iteration']['avg_launch_ms']*1e3,2), 'IL32', round(s['il_empc_step_cartpole_b32']['ms_per_step'],3), 'IL4096', round(s['il_empc_step_cartpole']['ms_per_step'],3), 'cimpl', round(s['config4_implicit_backward']['avg_ms'],4))

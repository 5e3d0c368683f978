import sys, json
sys.path.insert(0, '.')
import pktvisor_amd as pa
from tests.oracle_ctypes import load
o = load()
ALL = 0x3ff & ~8
names = ["cardinality","counters","quantiles","top_qtypes","top_rcodes","top_size","top_qnames","top_ports","xact_times"]
g = pa.pktvisor_reader('tests/golden/dns_ipv4_udp.pcap', periods=1, dns2_config={"enable": names})
r = o.run_file('tests/golden/dns_ipv4_udp.pcap', num_periods=1, window=1, dns2_groups=ALL)
print(json.dumps(g['1m']['dns']['unknown']['top_udp_ports_xacts']))
print(json.dumps(r['1m']['dns']['unknown']['top_udp_ports_xacts']))

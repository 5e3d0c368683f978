import sys, os
sys.path.insert(0, '.')
import pktvisor_amd as pa
from pktvisor_amd import synth
seed = int(sys.argv[1])
p = synth.tcp_dns_pcap(seed)
open('gpurun_out/tcp_seed.pcap', 'wb').write(p)
os.environ['PV_TCP_DUMP'] = 'gpurun_out/gpu_tcp_msgs.txt'
if os.path.exists('gpurun_out/gpu_tcp_msgs.txt'): os.remove('gpurun_out/gpu_tcp_msgs.txt')
out = pa.pktvisor_reader('gpurun_out/tcp_seed.pcap', host_spec='10.0.0.0/8,2001:db8::/32', periods=1)
print(out['1m']['dns']['wire_packets'])

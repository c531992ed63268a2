"""ProcessConnection (REMOTE_ADDR / REMOTE_PORT) and @ipMatch /
@ipMatchFromFile ([upstream coraza internal/operators/ipmatch.go:
net.ParseCIDR networks, net.ParseIP + IPNet.Contains]).  The oracle parses
addresses with Python's ipaddress, the device with its own Go-rule parser
(kernels.hip dev_parse_ip): the GPU test cross-checks the two."""
import pytest

import gpuinspect
import traffic
from oracle import compare, coraza

IPM = "127.0.0.1, 10.1.0.0/16,192.168.7.0/24 ,2001:db8::/32,::1, 10.300.0.0/16, bad, ::ffff:172.16.0.0/108, 1.2.3.4/033"

CASES = [("10.1.2.3", True), ("10.2.2.3", False), ("127.0.0.1", True), ("127.0.0.2", False), ("192.168.7.255", True),
         ("2001:db8:1::5", True), ("2001:db9::5", False), ("::1", True), ("::2", False), ("::ffff:10.1.9.9", True),
         ("172.16.4.4", True), ("172.32.0.1", False), ("172.31.0.1", True), ("010.1.2.3", False), ("10.1.2", False), ("", False),
         ("fe80::1%eth0", False), ("1.2.3.4", False), (" 10.1.2.3", False), ("2001:db8::1.2.3.4", True)]


@pytest.mark.parametrize("ip,want", CASES)
def test_oracle_ipmatch(ip, want):
    nets = coraza.ipmatch_networks(IPM)
    assert coraza.ipmatch(nets, ip.encode()) == want


RULES = """SecRuleEngine On
SecRule REMOTE_ADDR "@ipMatch %s" "id:1,phase:1,pass,setvar:tx.anomaly_score=+1"
SecRule REMOTE_ADDR "@ipMatchFromFile allow.txt" "id:2,phase:1,pass,setvar:tx.anomaly_score=+10"
SecRule ARGS:ip "@ipMatch %s" "id:3,phase:1,pass,setvar:tx.anomaly_score=+100"
SecRule REMOTE_PORT "@rx ^4[0-9]{3}$" "id:4,phase:1,pass,setvar:tx.anomaly_score=+1000"
SecRule REMOTE_ADDR "@rx ^10[.]" "id:5,phase:1,pass,setvar:tx.anomaly_score=+10000"
""" % (IPM, IPM)
FILES = {"allow.txt": b"# office\\n10.0.0.0/8\\r\\n\\n2001:db8::/32\\n"}


def test_compile_ipmatch():
    gpuinspect.Ruleset(RULES, data_files=FILES)
    coraza.parse_seclang(RULES, FILES)


@pytest.mark.gpu
def test_gpu_parity_connection_ipmatch():
    txs = []
    for k, (ip, _) in enumerate(CASES):
        t = gpuinspect.Transaction(method=b"GET", uri=b"/?ip=" + ip.replace(" ", "+").replace("%", "%25").encode())
        t.add_request_header("Host", "x")
        t.process_connection(ip, 4000 + 37 * k)
        txs.append(t)
    batch = gpuinspect.pack(txs)
    rs = gpuinspect.Ruleset(RULES, data_files=FILES)
    res = gpuinspect.Engine(rs).inspect(batch)
    cfg = coraza.parse_seclang(RULES, FILES)
    bad = compare.compare(res, compare.oracle_verdicts(cfg, batch, rs.exports))
    assert not bad, bad
    ai = list(gpuinspect.DEFAULT_EXPORTS).index("anomaly_score")
    assert [int(v["tx_export"][ai]) // 100 % 10 for v in res.verdicts] == [int(w) for _, w in CASES]
    big = traffic.TrafficGen(traffic.SEED + 17).batch(800)  # generator clients: IPv4 + IPv6
    res = gpuinspect.Engine(rs).inspect(big)
    bad = compare.compare(res, compare.oracle_verdicts(cfg, big, rs.exports))
    assert not bad, bad
    assert int((res.verdicts["tx_export"][:, ai] >= 10000).sum()) > 100

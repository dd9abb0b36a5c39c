"""Trace writer: bcsim_format_trace_line reproduces the
reference's NS_LOG_INFO text -- the original strings and Simulator::Now().
GetSeconds() streamed at the default ostream precision (6 significant digits).
Host code only (no GPU).  Expected strings are restated from the cited lines."""
import bcsim
from bcsim import _abi

TR = _abi.TR


def rec(kind, node, t_ns, a=0, b=0, c=0):
    return (0, t_ns, 0, 0, 0, node, kind, a, b, c)


def fmt(r, cfg=None):
    return bcsim.format_trace_line(r, cfg)


def test_pbft_lines(engine_lib):
    # pbft-node.cc:259 commit (global v, block_num, GetSeconds, values[block_num], "\n")
    assert fmt(rec(TR["PBFT_COMMIT"], 3, 158_176_006, a=1, b=7, c=9)) == \
        "node 3 在视图 1 中完成了第 7 次提交, 时间为 0.158176s, value is 9\n"
    # pbft-node.cc:387 leader broadcast, :408 stop, :278 view change (leader, then v)
    assert fmt(rec(TR["PBFT_BLOCK"], 0, 50_000_001, a=0, b=1)) == "主节点 node0开始广播区块, 时间为0.05s\n"
    assert fmt(rec(TR["PBFT_STOP"], 5, 2_000_000_040, a=40)) == " 已经发送了第 40个区块 at time: 2s"
    assert fmt(rec(TR["PBFT_VIEW"], 1, 3_050_000_000, a=2, b=1)) == "view-change完成, 当前主节点为 1视图为 2"


def test_raft_lines(engine_lib):
    # raft-node.cc:399 -- data = {'2', intToChar(m_id), <uninitialised, read as NUL>}
    assert fmt(rec(TR["RAFT_ELECTION"], 2, 177_000_005)) == "node2 start election: 22 at time: 0.177s"
    assert fmt(rec(TR["RAFT_LEADER"], 270, 158_176_006)) == "Node 270 become leader! at time 0.158176s"
    assert fmt(rec(TR["RAFT_BLOCK"], 270, 1_273_616_018, a=0)) == "At time 1.27362 leader处理完一个区块 0"
    assert fmt(rec(TR["RAFT_DONE"], 270, 3_700_000_000, a=50)) == "node270 已经处理完 50个区块 at time: 3.7s"
    assert fmt(rec(TR["RAFT_PROPOSAL"], 4, 1_158_176_026, a=3)) == "广播区块: 3, time: 1.15818 s"
    # :342 followed by :362 when round reaches 50
    assert fmt(rec(TR["RAFT_PROPOSAL"], 4, 3_608_176_026, a=49)) == \
        "广播区块: 49, time: 3.60818 s\nnode4 已经发送了 50个区块 at time: 3.60818s"
    # :122-123 StopApplication of the leader: two lines
    assert fmt(rec(TR["RAFT_STOP"], 4, 10_000_000_000, a=50, b=50)) == "Blocks:50 Rounds:50\nAt time 10 Stop"


def test_paxos_lines(engine_lib):
    assert fmt(rec(TR["PAXOS_COMMIT"], 0, 24_264_000, a=1)) == \
        "CLIENT COMMIT SUCCESS\n   ##clinet ticket##: 1 id: 0 at time: 0.024264s"
    # paxos-node.cc:518 -- data = {'0', intToChar(ticket), NUL}
    assert fmt(rec(TR["PAXOS_TICKET"], 1, 0, a=2)) == "node1 require_data: 02"


def test_compat_char_wraps(engine_lib):
    # intToChar(130) = '0' + 130 = 178 as a signed char: the byte 0xB2 is printed as is
    cfg = _abi.default_config(_abi.RAFT, 200)
    cfg.encoding = _abi.ENC_COMPAT
    line = fmt(rec(TR["RAFT_ELECTION"], 130, 150_000_006), cfg)
    assert line.encode("utf-8", errors="surrogateescape") == b"node130 start election: 2\xb2 at time: 0.15s"

"""RCCL's own account of a communicator (parallel/rccl_log.py): rank count and per-link
transport, parsed from NCCL_DEBUG=INFO lines, so a multi-GPU record can say whether N ranks
met over xGMI (P2P) or through host shared memory.  The lines below follow RCCL's INFO format
(``host:pid:tid [dev] NCCL INFO ...``); a 1-GPU box cannot produce peer links, so they are
written in that format rather than captured (parity unpinned)."""
import os

from terraform_provider_iterative_amd.parallel import rccl_log

XGMI_8 = [
    "node1:4242:4290 [0] NCCL INFO comm 0x55d5c1a0 rank 0 nRanks 8 nNodes 1 localRanks 8 "
    "localRank 0 MNNVL 0",
    "node1:4242:4290 [0] NCCL INFO Channel 00/32 :    0   1   2   3   4   5   6   7",
] + ["node1:4242:4290 [0] NCCL INFO Channel %02d/0 : 0[2a000] -> %d[%x000] via P2P/IPC comm "
     "0x55d5c1a0 nRanks 08" % (c, peer, 0x3a + peer) for c in range(2) for peer in range(1, 8)] + [
    "node1:4242:4290 [0] NCCL INFO Connected all rings, use ring PXN 0 GDR 1",
    "node1:4242:4290 [0] NCCL INFO comm 0x55d5c1a0 rank 0 nranks 8 cudaDev 0 busId 2a000 "
    "commId 0x1b2c - Init COMPLETE",
]


def test_eight_ranks_over_p2p():
    out = rccl_log.parse(XGMI_8)
    assert out["nranks"] == 8 and out["ranks_seen"] == [0]
    assert sorted(out["links"]) == ["0->%d" % p for p in range(1, 8)]
    assert out["transports"] == {"P2P/IPC": 7} and out["xgmi_only"] is True


def test_a_shared_memory_link_is_flagged():
    lines = XGMI_8 + ["node1:4242:4290 [0] NCCL INFO Channel 03/0 : 0[2a000] -> 5[da000] "
                      "via SHM/direct/direct"]
    out = rccl_log.parse(lines)
    assert out["links"]["0->5"] == "P2P/IPC+SHM/direct/direct"
    assert out["transports"]["SHM/direct/direct"] == 1 and out["xgmi_only"] is False


def test_nothing_logged_is_unknown_not_true():
    out = rccl_log.parse(["some unrelated line", "NCCL INFO Bootstrap : Using eth0"])
    assert out["nranks"] is None and out["links"] == {} and out["xgmi_only"] is None


def test_debug_env_and_files(tmp_path):
    env = rccl_log.debug_env(str(tmp_path / "rccl"), {"NCCL_DEBUG": "WARN"})
    assert env["NCCL_DEBUG"] == "WARN"  # what the caller set wins
    assert env["NCCL_DEBUG_FILE"].endswith("rccl-%p.log")
    path = tmp_path / "rccl" / ("rccl-%d.log" % os.getpid())
    path.write_text("\n".join(XGMI_8) + "\n")
    out = rccl_log.parse_files(str(tmp_path / "rccl" / "rccl-*.log"))
    assert out["files"] == 1 and out["nranks"] == 8 and out["xgmi_only"] is True

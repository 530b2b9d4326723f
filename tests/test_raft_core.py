"""Raft core under the deterministic simulator: election safety, log matching, leader
completeness, the current-term commit rule, persistence, snapshots -- and the concrete failures
the survey reproduced on the reference."""
import json
import os
import random

import pytest

from distributed_lms_raft_llm_amd.raft.core import (LEADER, NOOP_COMMAND, AppendRequest, Entry, NotLeader,
                                                    RaftConfig, RaftCore, VoteRequest)
from distributed_lms_raft_llm_amd.raft.sim import SimCluster
from distributed_lms_raft_llm_amd.raft.storage import FileStorage, MemoryStorage


def cmd(i):
    return json.dumps({"operation": "Register", "args": [f"user{i}", "pw", "student"]})


def user_cmds(seq):
    return [c for c in seq if c != NOOP_COMMAND]


@pytest.mark.parametrize("n", [1, 3, 5])
def test_elects_single_leader_fast(n):
    c = SimCluster(n, seed=n)
    lid = c.wait_leader(timeout=2.0)
    # randomized 150-300 ms timeouts: a leader within ~1 s (reference: ~91 s, Appendix A.4)
    assert c.now < 1.0
    c.run(1.0)
    assert c.leader() == lid
    c.check_safety()


def test_replicates_and_applies_on_every_node_including_first_entry():
    c = SimCluster(5, seed=1)
    c.wait_leader()
    for i in range(10):
        c.propose(cmd(i))
    c.run(0.5)
    for i in c.ids:
        # index-0 entry never committed in the reference (A.2); heartbeats carry commit (A.9)
        assert user_cmds(c.committed_on(i)) == [cmd(i) for i in range(10)]
    c.check_safety()


def test_leader_crash_reelects_and_keeps_committed_writes():
    c = SimCluster(5, seed=2)
    old = c.wait_leader()
    for i in range(5):
        c.propose(cmd(i))
    c.run(0.3)
    c.crash(old)
    t0 = c.now
    new = c.wait_leader(timeout=3.0)
    assert new != old
    assert c.now - t0 < 1.0  # reference failover: ~102 s
    c.propose(cmd(99))
    c.run(0.5)
    for i in c.ids:
        if i != old:
            assert user_cmds(c.committed_on(i)) == [cmd(i) for i in range(5)] + [cmd(99)]
    c.check_safety()


def test_exactly_quorum_alive_still_elects_and_commits():
    # reference: no leader within 100 s with 3 of 5 alive (Appendix A.5)
    c = SimCluster(5, seed=3)
    c.wait_leader()
    lid = c.leader()
    others = [i for i in c.ids if i != lid]
    c.crash(lid)
    c.crash(others[0])
    new = c.wait_leader(timeout=3.0)
    c.propose(cmd(1))
    c.run(0.5)
    alive = [i for i in c.ids if c.nodes[i].up]
    assert len(alive) == 3
    for i in alive:
        assert cmd(1) in c.committed_on(i)
    c.check_safety()


def test_minority_partition_cannot_commit_and_leader_steps_down():
    c = SimCluster(5, seed=4)
    lid = c.wait_leader()
    minority = [lid, [i for i in c.ids if i != lid][0]]
    majority = [i for i in c.ids if i not in minority]
    c.partition(minority, majority)
    idx7 = c.nodes[lid].core.propose(cmd(7), c.now)
    c.run(1.0)
    # (entries replicated to a majority before the cut, e.g. the no-op, may still commit)
    assert c.nodes[lid].core.commit_index < idx7
    # check-quorum: the isolated ex-leader stops claiming leadership
    assert c.nodes[lid].core.role != LEADER
    new = c.leader()
    assert new in majority
    c.propose(cmd(8))
    c.run(0.5)
    c.heal()
    c.run(1.5)
    for i in c.ids:
        seq = user_cmds(c.committed_on(i))
        assert cmd(8) in seq and cmd(7) not in seq  # the uncommitted minority write was overwritten
    c.check_safety()


def test_follower_rejects_client_writes():
    c = SimCluster(3, seed=5)
    lid = c.wait_leader()
    c.run(0.2)  # followers learn the leader from its first AppendEntries
    f = [i for i in c.ids if i != lid][0]
    with pytest.raises(NotLeader) as ei:
        c.nodes[f].core.propose(cmd(1), c.now)
    assert ei.value.leader_id == lid
    # and nothing was appended locally (reference A.7 left a dangling entry)
    assert all(e.command == NOOP_COMMAND for e in c.nodes[f].core.storage.entries(1, 100))


def test_vote_denied_to_stale_log_and_granted_once_per_term():
    st = MemoryStorage()
    core = RaftCore(1, [2, 3], st, now=0.0)
    st.append([Entry(1, "a"), Entry(2, "b")])
    st.save_meta(2, None)
    core.current_term = 2
    # candidate with a shorter/older log is refused
    r = core.step(VoteRequest(2, 1, 3, last_log_index=5, last_log_term=1), 0.0)[0]
    assert not r.granted and r.term == 3
    r = core.step(VoteRequest(3, 1, 3, last_log_index=2, last_log_term=2), 0.0)[0]
    assert r.granted
    # second candidate in the same term is refused
    r = core.step(VoteRequest(2, 1, 3, last_log_index=9, last_log_term=3), 0.0)[0]
    assert not r.granted
    assert st.load_meta() == (3, 3)


def test_append_conflict_truncates_and_stale_duplicate_does_not():
    st = MemoryStorage()
    core = RaftCore(2, [1, 3], st, now=0.0)
    st.append([Entry(1, "x1"), Entry(1, "x2"), Entry(2, "bad3"), Entry(2, "bad4")])
    core.current_term = 3
    st.save_meta(3, None)
    r = core.step(AppendRequest(1, 2, 3, 2, 1, [Entry(3, "y3")], leader_commit=3), 0.0)[0]
    assert r.success and r.index == 3
    assert [e.command for e in st.entries(1, 10)] == ["x1", "x2", "y3"]
    assert core.commit_index == 3
    # a delayed duplicate of an older, shorter append must not truncate
    r = core.step(AppendRequest(1, 2, 3, 1, 1, [Entry(1, "x2")], leader_commit=3), 0.0)[0]
    assert r.success
    assert [e.command for e in st.entries(1, 10)] == ["x1", "x2", "y3"]


def test_commit_only_counts_current_term_entries():
    # Raft Figure 8: an entry from an old term must not be committed by replica counting alone
    st = MemoryStorage()
    core = RaftCore(1, [2, 3, 4, 5], st, now=0.0)
    st.append([Entry(2, "old")])
    st.save_meta(4, None)
    core.current_term = 4
    core.role = LEADER
    for p in core.peers.values():
        p.match_index = 0
    core.peers[2].match_index = 1
    core.peers[3].match_index = 1
    core._advance_commit()
    assert core.commit_index == 0
    st.append([Entry(4, "new")])
    core.peers[2].match_index = 2
    core.peers[3].match_index = 2
    core._advance_commit()
    assert core.commit_index == 2


def test_persistence_across_restart(tmp_path):
    dirs = {i: str(tmp_path / f"n{i}") for i in (1, 2, 3)}
    c = SimCluster(3, seed=6, storage_factory=lambda i: FileStorage(dirs[i], fsync=False))
    c.wait_leader()
    for i in range(6):
        c.propose(cmd(i))
    c.run(0.5)
    term_before = {i: c.nodes[i].core.current_term for i in c.ids}
    for i in c.ids:
        c.crash(i)
        c.nodes[i].storage.close()
        c.nodes[i].storage = FileStorage(dirs[i], fsync=False)
        c.restart(i)
        assert c.nodes[i].core.current_term == term_before[i]
        assert c.nodes[i].core.last_index() >= 7
    c.wait_leader()
    c.propose(cmd(100))
    c.run(0.5)
    for i in c.ids:
        assert user_cmds(c.committed_on(i))[-1] == cmd(100)
    # the on-disk log is the reference's LogEntry format {"term", "command"} per line, plus the
    # entry's own index (crash-safe compaction)
    with open(os.path.join(dirs[1], "raft_log.jsonl")) as f:
        first = json.loads(f.readline())
    assert set(first) == {"term", "command", "index"} and first["index"] == 1
    c.check_safety()


def test_snapshot_install_for_lagging_follower():
    c = SimCluster(3, seed=7)
    lid = c.wait_leader()
    lag = [i for i in c.ids if i != lid][0]
    c.crash(lag)
    for i in range(30):
        c.propose(cmd(i))
    c.run(0.5)
    lc = c.nodes[lid].core
    lc.compact(lc.last_applied, json.dumps({"state": "snap"}))
    for p in c.ids:
        if p not in (lid, lag):
            c.nodes[p].core.compact(c.nodes[p].core.last_applied, json.dumps({"state": "snap"}))
    assert lc.storage.snapshot_meta()[0] > 0
    c.restart(lag)
    c.propose(cmd(999))
    c.run(1.0)
    core = c.nodes[lag].core
    assert core.storage.snapshot_meta()[0] >= lc.storage.snapshot_meta()[0]
    assert core.commit_index == lc.commit_index
    assert user_cmds(c.committed_on(lag))[-1] == cmd(999)


@pytest.mark.parametrize("seed", range(6))
def test_randomized_faults_preserve_safety(seed):
    rng = random.Random(seed)
    c = SimCluster(5, seed=seed, drop=0.05)
    c.wait_leader(timeout=5)
    proposed = 0
    for step in range(40):
        r = rng.random()
        if r < 0.1:
            victim = rng.choice(c.ids)
            if sum(n.up for n in c.nodes.values()) > 3:
                c.crash(victim)
        elif r < 0.25:
            for i, n in c.nodes.items():
                if not n.up:
                    c.restart(i)
        elif r < 0.3:
            ids = c.ids[:]
            rng.shuffle(ids)
            c.partition(ids[:2], ids[2:])
        elif r < 0.4:
            c.heal()
        if c.leader() is not None:
            try:
                c.propose(cmd(proposed))
                proposed += 1
            except NotLeader:
                pass
        c.run(rng.uniform(0.02, 0.3))
        c.check_safety()
    c.heal()
    for i, n in c.nodes.items():
        if not n.up:
            c.restart(i)
    c.run(3.0)
    c.check_safety()
    lid = c.wait_leader()
    c.propose(cmd(10_000))
    c.run(1.0)
    final = [user_cmds(c.committed_on(i)) for i in c.ids]
    assert all(f == final[0] for f in final)
    assert final[0][-1] == cmd(10_000)


def test_pre_vote_rejoining_node_does_not_disrupt_leader():
    """A follower cut off for many election timeouts keeps probing with pre-votes (its term never
    moves), and when it rejoins the healthy leader keeps its term and leadership (Raft thesis
    §9.6; without pre-vote the rejoining node's inflated term would force an election)."""
    c = SimCluster(5, seed=11)
    lid = c.wait_leader()
    term = c.nodes[lid].core.current_term
    victim = [i for i in c.ids if i != lid][0]
    c.partition([victim], [i for i in c.ids if i != victim])
    c.run(3.0)  # ~10-20 election timeouts on the victim
    assert c.nodes[victim].core.current_term == term
    assert c.nodes[victim].core.stats.elections_started == 0
    c.heal()
    c.run(1.0)
    assert c.leader() == lid and c.nodes[lid].core.current_term == term
    assert c.nodes[victim].core.leader_id == lid
    c.check_safety()


def test_pre_vote_is_side_effect_free_and_lease_refuses():
    st = MemoryStorage()
    core = RaftCore(1, [2, 3], st, now=0.0)
    st.append([Entry(1, "a")])
    st.save_meta(1, None)
    core.current_term = 1
    # no leader heard: a pre-vote for term 2 with an up-to-date log is granted, nothing persists
    r = core.step(VoteRequest(2, 1, 2, last_log_index=1, last_log_term=1, pre=True), 1.0)[0]
    assert r.granted and r.pre and r.term == 2
    assert st.load_meta() == (1, None) and core.current_term == 1
    # stale log: refused
    r = core.step(VoteRequest(3, 1, 2, last_log_index=0, last_log_term=0, pre=True), 1.0)[0]
    assert not r.granted
    # after hearing from the leader of term 1, both pre-votes and real votes are refused in the lease
    core.step(AppendRequest(3, 1, 1, 1, 1, [], 1), 2.0)
    r = core.step(VoteRequest(2, 1, 2, last_log_index=1, last_log_term=1, pre=True), 2.05)[0]
    assert not r.granted
    r = core.step(VoteRequest(2, 1, 2, last_log_index=1, last_log_term=1), 2.05)[0]
    assert not r.granted and core.current_term == 1
    # once the lease lapsed, the real vote goes through
    r = core.step(VoteRequest(2, 1, 2, last_log_index=1, last_log_term=1), 2.5)[0]
    assert r.granted and core.current_term == 2


def test_stale_append_never_moves_commit_index_back():
    """A duplicate / reordered AppendEntries with a short ``last_new`` must not regress the
    follower's commit index."""
    from distributed_lms_raft_llm_amd.raft.core import AppendRequest, Entry, RaftCore

    core = RaftCore(2, [1, 3], MemoryStorage())
    ents = [Entry(1, f"c{i}") for i in range(5)]
    r = core.step(AppendRequest(1, 2, 1, 0, 0, ents, 5), 0.0)[0]
    assert r.success and core.commit_index == 5
    # the stale first AppendEntries (one entry, leader_commit 3) arrives late
    r = core.step(AppendRequest(1, 2, 1, 0, 0, ents[:1], 3), 0.01)[0]
    assert r.success and core.commit_index == 5 and core.last_index() == 5
    r = core.step(AppendRequest(1, 2, 1, 0, 0, ents[:2], 9), 0.02)[0]
    assert core.commit_index == 5  # min(leader_commit, last_new) = 2 < 5


def test_crash_between_snapshot_and_log_rewrite(tmp_path):
    """Compaction replaces the snapshot, then rewrites the log; a crash in between leaves the OLD
    log.  Its entries carry their own indices, so loading drops the snapshotted prefix instead of
    shifting every entry to the wrong index."""
    from distributed_lms_raft_llm_amd.raft.core import Entry

    d = str(tmp_path / "n")
    st = FileStorage(d, fsync=False)
    st.append([Entry(1, f"c{i}") for i in range(1, 11)])  # indices 1..10
    old_log = open(os.path.join(d, "raft_log.jsonl")).read()
    st.compact(6, 1, "state@6")
    st.close()
    with open(os.path.join(d, "raft_log.jsonl"), "w") as f:  # crash: the log rewrite never happened
        f.write(old_log)
    st2 = FileStorage(d, fsync=False)
    assert st2.snapshot_meta() == (6, 1) and st2.last_index() == 10
    assert [e.command for e in st2.entries(7, 11)] == ["c7", "c8", "c9", "c10"]
    st2.append([Entry(2, "c11")])
    st2.close()
    st3 = FileStorage(d, fsync=False)
    assert st3.last_index() == 11 and st3.entries(11, 12)[0].command == "c11" and st3.term_at(11) == 2
    # round-1 logs (no index field) still load sequentially after the snapshot
    with open(os.path.join(d, "raft_log.jsonl"), "w") as f:
        for i in range(7, 9):
            f.write(json.dumps({"term": 1, "command": f"c{i}"}) + "\n")
    st4 = FileStorage(d, fsync=False)
    assert st4.last_index() == 8 and st4.entries(7, 9)[1].command == "c8"

"""Lachesis self-learning placement: history recording, rule-based and learned key choice, and
co-partitioning by the advised key (reference: src/selfLearning, RuleBasedDataPlacementOptimizerForLoadJob)."""
import torch

from netsdb_amd.client import PDBClient
from netsdb_amd.computations import ScanSet, WriteSet
from netsdb_amd.objects.builtin import Employee
from netsdb_amd.selflearning import LearnedAdvisor, SelfLearningDB
from tests.test_engine import Dept, EmpDept, EmpJoinDept, SalaryByDept, _emps


def test_rule_based_advice(tmp_path):
    c = PDBClient(root=str(tmp_path), broadcast_threshold=0)
    hook = c.enable_self_learning()
    c.create_database("db")
    c.create_set("db", "emps", Employee)
    c.send_data("db", "emps", _emps())
    c.create_set("db", "depts", Dept)
    c.send_data("db", "depts", [Dept("eng", 1)])
    for _ in range(2):
        j = EmpJoinDept()
        j.set_input(0, ScanSet("db", "emps", Employee))
        j.set_input(1, ScanSet("db", "depts", Dept))
        c.create_set("db", "out", EmpDept)
        c.execute_computations(WriteSet("db", "out").set_input(j))
    c.create_set("db", "tot", None)
    c.execute_computations(WriteSet("db", "tot").set_input(SalaryByDept().set_input(ScanSet("db", "emps", Employee))))
    assert hook.advisor.best_key("db", "emps") == ("att", "department")
    assert hook.advisor.best_key("db", "depts") == ("att", "name")
    # method keys are learned too (aggregate used getDepartment)
    assert ("method", "getDepartment") in [(k, n) for k, n, _ in hook.db.candidates("db", "emps")]
    # policy='auto' consults the advisor; the policy hashes by department
    c.remove_set("db", "emps")                       # reload the set: placement from history
    c.create_set("db", "emps", Employee, policy="auto")
    pol = c.policies[("db", "emps")]
    from netsdb_amd.objects.record import RecordBatch

    b = RecordBatch.from_objects(_emps(8))
    d = pol.assign(b, 4)
    depts = [e.department for e in _emps(8)]
    for i in range(8):
        for j in range(8):
            if depts[i] == depts[j]:
                assert d[i] == d[j]


def test_learned_advisor_prefers_faster_key():
    db = SelfLearningDB()
    for k, secs in (("a", 5.0), ("b", 1.0)):
        db.record_placement("d", "s", ("att", k))
        db.record_job("j", secs, [{"db": "d", "set": "s", "sink": "Shuffle", "comp": "C", "key": ("att", "a"), "index": 0},
                                   {"db": "d", "set": "s", "sink": "Shuffle", "comp": "C", "key": ("att", "b"), "index": 0}])
    adv = LearnedAdvisor(db, epsilon=0.0)
    assert adv.best_key("d", "s") == ("att", "b")


def test_drl_advisor_learns_faster_placement(tmp_path):
    """DRLBasedDataPlacementOptimizer parity: the Q-network agent, fed the consumer-job time of each
    placement it chooses, converges to the placement under which the consumers run faster."""
    from netsdb_amd.selflearning import DRLAdvisor

    db = SelfLearningDB()
    uses = [{"db": "d", "set": "s", "sink": "Shuffle", "comp": "J", "key": ("att", k), "index": 0} for k in ("a", "b")]
    db.record_job("warm", 1.0, uses)                          # both keys are candidates
    adv = DRLAdvisor(db, epsilon=0.2, seed=3)
    rnd = torch.Generator().manual_seed(0)
    picks = []
    for _ in range(80):
        k = adv.best_key("d", "s")
        db.record_placement("d", "s", k)
        # environment: co-partitioning on 'b' makes the consumer job ~3x faster
        secs = (1.0 if k[1] == "b" else 3.0) + 0.1 * float(torch.rand(1, generator=rnd))
        db.record_job("consumer", secs, uses)
        adv.observe("d", "s", k[1], secs)
        picks.append(k[1])
    adv.epsilon = 0.0
    assert adv.best_key("d", "s") == ("att", "b")
    assert picks[-30:].count("b") >= 20
    path = str(tmp_path / "q.pt")
    adv.save(path)
    adv2 = DRLAdvisor(db, epsilon=0.0, seed=9)
    adv2.load(path)
    assert adv2.best_key("d", "s") == ("att", "b")


def test_drl_hook_through_engine(tmp_path):
    """enable_self_learning(learned="drl"): jobs feed the agent, policy='auto' asks it for the key."""
    c = PDBClient(root=str(tmp_path), broadcast_threshold=0)
    hook = c.enable_self_learning(learned="drl")
    c.create_database("db")
    c.create_set("db", "emps", Employee)
    c.send_data("db", "emps", _emps())
    c.create_set("db", "depts", Dept)
    c.send_data("db", "depts", [Dept("eng", 1)])
    for _ in range(3):
        j = EmpJoinDept()
        j.set_input(0, ScanSet("db", "emps", Employee))
        j.set_input(1, ScanSet("db", "depts", Dept))
        c.create_set("db", "out", EmpDept)
        c.execute_computations(WriteSet("db", "out").set_input(j))
        c.remove_set("db", "depts")
        c.create_set("db", "depts", Dept, policy="auto")      # placement chosen by the agent, then rewarded
        c.send_data("db", "depts", [Dept("eng", 1)])
    assert c.policies[("db", "depts")] is not None
    assert len(hook.advisor.replay) >= 1

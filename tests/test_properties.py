"""Property-based tests (hypothesis) for the native core and the cluster emulation.

* the C++ JSON codec round-trips arbitrary documents exactly (int64, unicode, nesting);
* the C++ work queue keeps client-go's invariants for arbitrary add/get/done sequences:
  a key is never handed out twice while processing, adds while processing are not lost,
  and duplicates collapse;
* the fake API server's label-selector matcher agrees with a direct reference
  implementation for arbitrary label sets and equality/inequality/existence selectors;
* reconcile is a pure function: the same input always yields the same actions, and the
  number of pods it creates never exceeds the replica count for any set of existing pods.
"""
import json

from hypothesis import given, settings
from hypothesis import strategies as st

from opfixtures import new_job, opcore, reconcile
from pytorch_operator_amd.cluster.fake_apiserver import label_selector_matches

json_scalars = st.one_of(st.none(), st.booleans(), st.integers(min_value=-(2 ** 63), max_value=2 ** 63 - 1),
                         st.text(max_size=12))
json_docs = st.recursive(json_scalars, lambda ch: st.one_of(st.lists(ch, max_size=4),
                                                             st.dictionaries(st.text(max_size=6), ch, max_size=4)),
                         max_leaves=20)


@settings(max_examples=150, deadline=None)
@given(json_docs)
def test_json_roundtrip_exact(doc):
    text = json.dumps(doc)
    assert json.loads(opcore().json_roundtrip(text)) == doc


ops = st.lists(st.tuples(st.sampled_from(["add", "get", "done"]), st.sampled_from(["a", "b", "c", "d"])),
               max_size=40)


@settings(max_examples=150, deadline=None)
@given(ops)
def test_workqueue_invariants(seq):
    q = opcore().WorkQueue()
    processing, pending_model = set(), []
    dirty = set()
    for op, key in seq:
        if op == "add":
            q.add(key)
            if key not in dirty:
                dirty.add(key)
                if key not in processing:
                    pending_model.append(key)
        elif op == "get":
            got = q.get(0.0)
            if pending_model:
                exp = pending_model.pop(0)
                assert got == exp
                assert got not in processing
                processing.add(got)
                dirty.discard(got)
            else:
                assert got in (None, "")
        else:
            if key in processing:
                q.done(key)
                processing.discard(key)
                if key in dirty:
                    pending_model.append(key)
        assert q.len() == len(pending_model)


labels = st.dictionaries(st.sampled_from(["app", "role", "tier", "x"]), st.sampled_from(["a", "b", "c"]), max_size=4)
terms = st.lists(st.tuples(st.sampled_from(["=", "!=", "exists", "!exists"]), st.sampled_from(["app", "role", "tier", "x"]),
                           st.sampled_from(["a", "b", "c"])), max_size=3)


@settings(max_examples=300, deadline=None)
@given(labels, terms)
def test_label_selector_matches_reference(lab, ts):
    parts, expect = [], True
    for op, k, v in ts:
        if op == "=":
            parts.append(f"{k}={v}")
            expect &= lab.get(k) == v
        elif op == "!=":
            parts.append(f"{k}!={v}")
            expect &= lab.get(k) != v
        elif op == "exists":
            parts.append(k)
            expect &= k in lab
        else:
            parts.append(f"!{k}")
            expect &= k not in lab
    assert label_selector_matches(",".join(parts), lab) == expect


phases = st.sampled_from(["Pending", "Running", "Succeeded", "Failed"])


@settings(max_examples=60, deadline=None)
@given(st.integers(min_value=0, max_value=4), st.lists(st.tuples(st.sampled_from(["master", "worker"]),
                                                                 st.integers(min_value=0, max_value=5), phases),
                                                       max_size=6))
def test_reconcile_is_pure_and_bounded(workers, pods_desc):
    from opfixtures import new_pod
    job = new_job(workers)
    pods = [new_pod(job, rt, idx, phase) for rt, idx, phase in pods_desc]
    now = 1_700_000_000_000
    r1 = reconcile(job, pods=pods, now_ms=now)
    r2 = reconcile(job, pods=pods, now_ms=now)
    assert json.dumps(r1, sort_keys=True) == json.dumps(r2, sort_keys=True)
    assert len(r1.get("createPods") or []) <= 1 + workers

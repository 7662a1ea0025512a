"""Lazy synthetic image names (serving/jobs.SynthNames): a synthetic job is two integers in the
replicated log and in every batch — slicing, iteration, equality with plain lists, the JSON
round trip of a submit record and of a queue snapshot, and the replica applying it."""
import json

from distributed_machine_learning_amd.parallel.rank_backend import synthetic_names
from distributed_machine_learning_amd.parallel.service import ReplicatedCoordinator
from distributed_machine_learning_amd.serving.jobs import (Batch, JobManager, SynthNames, as_names, json_default,
                                                           make_batches)


def test_sequence_behaviour():
    s = synthetic_names(10)
    assert isinstance(s, SynthNames) and len(s) == 10
    assert list(s) == [f"synthetic:{i}" for i in range(10)]
    assert s[0] == "synthetic:0" and s[-1] == "synthetic:9"
    assert s[2:5] == ["synthetic:2", "synthetic:3", "synthetic:4"] and isinstance(s[2:5], SynthNames)
    assert s[::3] == ["synthetic:0", "synthetic:3", "synthetic:6", "synthetic:9"]
    assert s[8:20] == ["synthetic:8", "synthetic:9"] and len(s[20:30]) == 0
    assert s == [f"synthetic:{i}" for i in range(10)] and s != ["synthetic:0"]


def test_batches_stay_lazy_and_match_the_list_form():
    lazy = make_batches(31, "ResNet50", synthetic_names(1000), 256)
    eager = make_batches(31, "ResNet50", [f"synthetic:{i}" for i in range(1000)], 256)
    assert [len(b.images) for b in lazy] == [256, 256, 256, 232]
    assert all(isinstance(b.images, SynthNames) for b in lazy)
    assert [list(b.images) for b in lazy] == [b.images for b in eager]


def test_json_round_trips():
    rec = {"op": "submit", "model": "ResNet50", "images": synthetic_names(2_457_600), "job_id": 31}
    wire = json.dumps([rec], default=json_default)
    assert len(wire) < 200   # 9,600 batches of 256 names: two integers on the wire
    back = json.loads(wire)[0]
    assert as_names(back["images"]) == SynthNames(0, 2_457_600)
    b = Batch(31, 2, "ResNet50", synthetic_names(512)[256:512])
    d = json.loads(json.dumps(b.to_dict()))
    assert Batch.from_dict(d).images == b.images and Batch.from_dict(d).key == (31, 2)
    jm = JobManager({"ResNet50": 256, "InceptionV3": 128})
    jm.submit_images("ResNet50", synthetic_names(600), "t")
    snap = json.loads(json.dumps(jm.snapshot()))
    jm2 = JobManager({"ResNet50": 256, "InceptionV3": 128})
    jm2.restore(snap)
    assert [list(b.images) for b in jm2.queues["ResNet50"]] == [list(b.images) for b in jm.queues["ResNet50"]]


def test_replica_applies_the_compact_record():
    a = ReplicatedCoordinator({"ResNet50": 256, "InceptionV3": 128}, cap=256)
    b = ReplicatedCoordinator({"ResNet50": 256, "InceptionV3": 128}, cap=256)
    rec = {"op": "submit", "model": "ResNet50", "images": synthetic_names(256 * 40), "job_id": a.next_job_id()}
    ra = a.apply(rec)                                                    # the coordinator: the object
    rb = b.apply(json.loads(json.dumps(rec, default=json_default)))      # a replica: the wire form
    assert ra == rb == {"jobid": 31, "batches": 40}
    qa, qb = a.jobs.queues["ResNet50"], b.jobs.queues["ResNet50"]
    assert [x.key for x in qa] == [x.key for x in qb] and list(qa[7].images) == list(qb[7].images)

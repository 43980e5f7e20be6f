"""Generates the committed fixtures under tests/golden/.  Re-run with
`python tests/golden/make_golden.py` (needs oracle/liboracle.so, built by make).

1. reference_known_answers.json — the reference's OWN known answers, written out
   as data with their file:line: the storage unit tests, the range-partition
   unit tests, and the reference probe outputs recorded in SURVEY.md §0 (the
   survey compiled the reference storages and ran them).  These pin the oracle.
2. assign_vectors.npz — regression vectors for the assign path produced by the
   oracle's MapStorageRef restatement (uniform / Zipf duplicates, sorted runs,
   keys >= 2^31, missing-key Gets, ragged and empty batches; int32 / float32 /
   float64).  tests/test_oracle.py re-derives them with BOTH restatements
   (MapStorageRef and VectorStorageRef) and the GPU tests replay them.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))

KNOWN = {
    "note": "Known answers of the reference (tkwong/parameter_server). Data only.",
    "storage_cases": [
        {
            "name": "AddGetInt",
            "cite": "server/vector_storage_test.cpp:19-43, server/map_storage_test.cpp:19-43",
            "dtype": "int32",
            "ops": [["add", [13, 14, 15], [1, 2, 3]], ["get", [13, 14, 15], [1, 2, 3]]],
        },
        {
            "name": "AddGetFloat",
            "cite": "server/vector_storage_test.cpp:45-66, server/map_storage_test.cpp:45-66",
            "dtype": "float32",
            "ops": [["add", [13, 14, 15], [0.1, 0.2, 0.3]], ["get", [13, 14, 15], [0.1, 0.2, 0.3]]],
        },
        {
            "name": "SubAddSubGet",
            "cite": "server/vector_storage_test.cpp:68-78, server/map_storage_test.cpp:68-75",
            "dtype": "float32",
            "ops": [["add", [13, 14, 15], [0.1, 0.2, 0.3]], ["get", [13, 14, 15], [0.1, 0.2, 0.3]]],
        },
        {
            "name": "LastWriteWinsProbe",
            "cite": "SURVEY.md §0.1 (probe of server/map_storage.hpp and server/vector_storage.hpp: "
                    "Add{5:1,5:2,7:3}; Add{7:10}; Get{5,7,9} -> {2,10,0} for both storages)",
            "dtype": "int32",
            "ops": [["add", [5, 5, 7], [1, 2, 3]], ["add", [7], [10]], ["get", [5, 7, 9], [2, 10, 0]]],
        },
        {
            "name": "LastWriteWinsProbeFloat",
            "cite": "SURVEY.md §0.1 (same probe, float values)",
            "dtype": "float32",
            "ops": [["add", [5, 5, 7], [1, 2, 3]], ["add", [7], [10]], ["get", [5, 7, 9], [2, 10, 0]]],
        },
    ],
    "model_cases": [
        {
            "name": "SSP CheckGetAndAdd",
            "cite": "server/consistency/ssp_model_test.cpp:29-117",
            "staleness": 1, "tids": [2, 3],
            "ops": [["add", 2, [0], [1]], ["add", 3, [1], [2]], ["get", 2, [0]], ["get", 3, [1]]],
            "replies": [{"recver": 2, "sender": 0, "keys": [0], "vals": [1]},
                        {"recver": 3, "sender": 0, "keys": [1], "vals": [2]}],
        },
        {
            "name": "BSP CheckGetAndAdd",
            "cite": "server/consistency/bsp_model_test.cpp:29-130",
            "tids": [2, 3],
            "ops": [["get", 2, [1]], ["add", 2, [1], [100]], ["clock", 2], ["get", 3, [1]],
                    ["clock", 3], ["get", 3, [1]]],
            "replies": [{"recver": 2, "keys": [1], "vals": [0]},
                        {"recver": 3, "keys": [1], "vals": [0]},
                        {"recver": 3, "keys": [1], "vals": [100]}],
        },
        {
            "name": "SSP CheckStaleness",
            "cite": "server/consistency/ssp_model_test.cpp:161-251",
            "staleness": 2, "tids": [2, 3],
            # worker 2 runs ahead: its Get at clock 3 > min 0 + 2 is buffered at
            # 3 - 2 = 1 and released (as the request) when worker 3 clocks
            "ops": [["get", 2, [0]], ["clock", 2], ["add", 2, [0], [1]], ["clock", 2], ["clock", 2],
                    ["get", 2, [0]], ["pending", 1, 1], ["clock", 3], ["get", 2, [0]], ["pending", 1, 0]],
        },
        {
            "name": "ASP CheckGetAndAdd",
            "cite": "server/consistency/asp_model_test.cpp:33-179",
            "tids": [2, 3],
            # Gets are served at once, in order with the Adds; Clock is a no-op
            "ops": [["get", 2, [0]], ["get", 3, [1]], ["get", 3, [1]], ["add", 2, [1], [1]],
                    ["clock", 2], ["get", 2, [1]], ["add", 3, [0], [1]], ["clock", 3], ["get", 3, [0]]],
            "replies": [{"recver": 2, "sender": 0, "keys": [0], "vals": [0]},
                        {"recver": 3, "sender": 0, "keys": [1], "vals": [0]},
                        {"recver": 3, "sender": 0, "keys": [1], "vals": [0]},
                        {"recver": 2, "sender": 0, "keys": [1], "vals": [1]},
                        {"recver": 3, "sender": 0, "keys": [0], "vals": [1]}],
        },
    ],
    # Cases the reference leaves undefined, pinned to the restatement's choice
    # (DESIGN.md §6 "BSP re-buffered Get"); not reference known answers
    "restatement_cases": [
        {
            "name": "BSP Get two clocks ahead is re-buffered",
            "cite": "server/consistency/bsp_model.cpp:14-31 (deviation, DESIGN.md §6)",
            "tids": [2, 3],
            # worker 2 runs two clocks ahead and Gets; worker 3's first clock
            # advances the min clock to 1 and flushes the Add, but worker 2
            # (progress 2) is still ahead: the released Get is buffered again.
            # The reference iterates get_buffer_ while this->Get pushes back
            # into it and then clear()s it: the Get is dropped (undefined
            # behaviour if the push_back reallocates) and worker 2 waits for
            # ever.  The restatement keeps it and answers it at the next
            # advance, with the value the flushed Add wrote.
            "ops": [["clock", 2], ["clock", 2], ["add", 2, [1], [7]], ["get", 2, [1]], ["pending_get", 1],
                    ["clock", 3], ["pending_get", 1], ["replies", 0], ["clock", 3], ["pending_get", 0]],
            "replies": [{"recver": 2, "keys": [1], "vals": [7]}],
            "reference_behaviour": "dropped after the first advance (get_buffer_.clear()); never answered",
        },
    ],
    # server/util: the progress tracker and pending buffer the SSP/BSP models
    # are built on.  ops: [query, argument(s), expected]
    "util_cases": [
        {"name": "ProgressTracker Basic", "cite": "server/util/progress_tracker_test.cpp:19-25", "tids": [2, 7],
         "ops": [["num_threads", 2], ["progress", 2, 0], ["progress", 7, 0]]},
        {"name": "ProgressTracker CheckThreadValid", "cite": "server/util/progress_tracker_test.cpp:27-34",
         "tids": [2, 7], "ops": [["valid", 2, True], ["valid", 3, False], ["valid", 6, False], ["valid", 7, True]]},
        {"name": "ProgressTracker Advance", "cite": "server/util/progress_tracker_test.cpp:36-47", "tids": [2, 7],
         "ops": [["min_clock", 0], ["advance", 2, -1], ["advance", 7, 1], ["advance", 7, -1], ["advance", 7, -1],
                 ["advance", 2, 2], ["progress", 2, 2], ["progress", 7, 3]]},
        {"name": "ProgressTracker UniqueMin", "cite": "server/util/progress_tracker_test.cpp:49-55", "tids": [2, 7],
         "ops": [["unique_min", 2, False], ["advance", 2, -1], ["unique_min", 7, True]]},
        {"name": "PendingBuffer PushAndPop", "cite": "server/util/pending_buffer_test.cpp:21-61",
         "ops": [["push", 0], ["push", 0], ["push", 1], ["size", 0, 2], ["size", 1, 1], ["pop", 0, 2],
                 ["pop", 1, 1]]},
        # server/server_thread.cpp's dispatch (the path's caller)
        {"name": "ServerThread RegisterModel", "cite": "server/server_thread_test.cpp:35-43",
         "ops": [["register", 0], ["model_not_null", 0]]},
        {"name": "ServerThread Clock", "cite": "server/server_thread_test.cpp:45-66",
         "ops": [["push", "clock"], ["push", "clock"], ["exit"], ["count", "clock", 2]]},
        {"name": "ServerThread Add", "cite": "server/server_thread_test.cpp:68-89",
         "ops": [["push", "add"], ["exit"], ["count", "add", 1]]},
        {"name": "ServerThread Get", "cite": "server/server_thread_test.cpp:91-114",
         "ops": [["push", "get"], ["push", "get"], ["push", "get"], ["exit"], ["count", "get", 3]]},
        # worker/callback_runner.cpp: where a worker's Get collects its replies
        # (SURVEY §8 a12's producer side)
        {"name": "CallbackRunner AddResponse", "cite": "worker/callback_runner_test.cpp:19-57",
         "replies": [[[3], [0.1]], [[4, 5, 6], [0.4, 0.2, 0.3]]],
         "expect": {"reply": {"3": 0.1, "4": 0.4, "5": 0.2, "6": 0.3}, "finished": True}},
        {"name": "CallbackRunner AddResponseTwoWorkers", "cite": "worker/callback_runner_test.cpp:59-108",
         "replies": [[[3], [0.1]], [[4, 5, 6], [0.4, 0.2, 0.3]]],
         "expect": {"worker0_reply": {"3": 0.1, "4": 0.4, "5": 0.2, "6": 0.3}, "worker1_sum": 1.0}},
    ],
    "slice_cases": [
        {"cite": "base/range_partition_manager_test.cpp:19-33", "ranges": [[2, 4], [4, 7], [7, 10]],
         "keys": [2, 8, 9], "expect": [[0, [2]], [2, [8, 9]]]},
        {"cite": "base/range_partition_manager_test.cpp:35-56", "ranges": [[0, 4], [4, 8], [8, 10]],
         "keys": [2, 5, 9], "expect": [[0, [2]], [1, [5]], [2, [9]]]},
        {"cite": "SURVEY.md §0.4 probe (unsorted input misroutes)", "ranges": [[0, 4], [4, 8], [8, 12]],
         "keys": [5, 1, 9], "expect": [[1, [5]], [2, [1, 9]]]},
        {"cite": "SURVEY.md §0.4 probe (beyond every range -> last server)",
         "ranges": [[0, 4], [4, 8], [8, 12]], "keys": [3, 20], "expect": [[0, [3]], [2, [20]]]},
        {"cite": "SURVEY.md §0.4 probe (below the first range -> last server)",
         "ranges": [[2, 4], [4, 8]], "keys": [0, 5], "expect": [[1, [0, 5]]]},
        {"cite": "empty input", "ranges": [[0, 4], [4, 8]], "keys": [], "expect": []},
    ],
    # ConsistentHashingPartitionManager (the Engine's default partitioner): the
    # slices its own test asserts, with the per-key servers its recorded log
    # lines give (server ids [0, 1, 2]); slices in first-appearance order
    "hash_slice_cases": [
        {"cite": "base/consistent_hashing_partition_manager_test.cpp:48-77", "servers": [0, 1, 2],
         "keys": [2, 8, 9], "expect": [[0, [2, 8]], [2, [9]]]},
        {"cite": "base/consistent_hashing_partition_manager_test.cpp:79-106", "servers": [0, 1, 2],
         "keys": [2, 8, 9, 10, 11, 12, 13], "expect": [[0, [2, 8, 13]], [2, [9, 10, 11]], [1, [12]]]},
        {"cite": "base/consistent_hashing_partition_manager_test.cpp:109-139 (SliceKVs)", "servers": [0, 1, 2],
         "keys": [2, 5, 9], "vals": [0.2, 0.5, 0.9],
         "expect": [[0, [2], [0.2]], [1, [5], [0.5]], [2, [9], [0.9]]]},
        {"cite": "empty input", "servers": [0, 1, 2], "keys": [], "expect": []},
    ],
}

DT = {"int32": np.int32, "float32": np.float32, "float64": np.float64}


def gen_vectors(oracle):
    rng = np.random.default_rng(20261015)
    out = {}
    cases = []
    for dname, dt in DT.items():
        for dist in ("uniform", "zipf", "sorted_runs", "high_keys"):
            name = f"{dist}_{dname}"
            ref = oracle.MapStorageRef(dt)
            sizes = [1024, 1, 0, 999, 1536]
            for j, n in enumerate(sizes):
                if dist == "uniform":
                    k = rng.integers(0, 3000, size=n)
                elif dist == "zipf":
                    k = (rng.zipf(1.3, size=n) * 7919) % 5000
                elif dist == "sorted_runs":
                    k = np.sort(rng.integers(100, 900, size=n))
                else:
                    k = rng.integers(2**31 - 500, 2**31 + 500, size=n)
                k = k.astype(np.uint32)
                if dt is np.int32:
                    v = rng.integers(-2**31, 2**31 - 1, size=n, dtype=np.int64).astype(np.int32)
                else:
                    v = rng.standard_normal(n).astype(dt)
                out[f"{name}/add{j}/keys"] = k
                out[f"{name}/add{j}/vals"] = v
                ref.add(k, v)
            q = np.concatenate([rng.integers(0, 5000, size=1200),
                                rng.integers(2**31 - 600, 2**31 + 600, size=400),
                                rng.integers(0, 2**32, size=96)]).astype(np.uint32)
            out[f"{name}/get/keys"] = q
            out[f"{name}/get/expect"] = ref.get(q)
            cases.append({"name": name, "dtype": dname, "n_adds": len(sizes)})
    return out, cases


def main():
    import oracle

    oracle.build()
    with open(os.path.join(HERE, "reference_known_answers.json"), "w") as f:
        json.dump(KNOWN, f, indent=1)
    arrays, cases = gen_vectors(oracle)
    np.savez_compressed(os.path.join(HERE, "assign_vectors.npz"), **arrays)
    with open(os.path.join(HERE, "assign_vectors.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (oracle MapStorageRef)", "cases": cases}, f,
                  indent=1)
    print("wrote", len(arrays), "arrays")


if __name__ == "__main__":
    main()

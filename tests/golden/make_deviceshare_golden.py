"""Transcribe the reference DeviceShare tests' known-answer cases into
tests/golden/deviceshare_cases.json (data only: inputs and expected outputs,
each with its source file:line; quantities as integers: Gi = 2^30 bytes).

Paths relative to pkg/scheduler/plugins/deviceshare/.  Node device state is
given as per-minor (total, used) per type; the tests that set deviceFree
directly set it to total - used, which is what the engine derives.
Run: python tests/golden/make_deviceshare_golden.py
"""
import json
import os

GI = 1 << 30
GPU = lambda core, ratio, mem: {"gpu-core": core, "gpu-memory-ratio": ratio, "gpu-memory": mem}


def node(gpu=None, rdma=None, fpga=None, present=True):
    """{type: [(minor, total, used)]}"""
    return {"present": present, "gpu": gpu or [], "rdma": rdma or [], "fpga": fpga or []}


CASES = {
    # scoring_test.go TestScore (node score, default LeastAllocated over
    # gpu-memory-ratio / rdma / fpga; MostAllocated where named)
    "score": [
        {"src": "scoring_test.go:101-136", "name": "completely idle node",
         "req": {"gpu-core": 100, "gpu-memory-ratio": 100},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(0, 0, 0))]), "want": 0},
        {"src": "scoring_test.go:138-183", "name": "multiple GPU devices and completely idle",
         "req": {"gpu-core": 50, "gpu-memory-ratio": 50},
         "node": node(gpu=[(0, GPU(400, 400, 64 * GI), GPU(0, 0, 0)), (1, GPU(400, 400, 64 * GI), GPU(0, 0, 0))]),
         "want": 93},
        {"src": "scoring_test.go:185-229", "name": "remaining device resources",
         "req": {"gpu-core": 50, "gpu-memory-ratio": 50},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(25, 25, 4 * GI))]), "want": 25},
        {"src": "scoring_test.go:231-276", "name": "remaining device resources with MostAllocated strategy",
         "most": True, "req": {"gpu-core": 50, "gpu-memory-ratio": 50},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(25, 25, 4 * GI))]), "want": 75},
        {"src": "scoring_test.go:278-338", "name": "requested multiple resources on the remaining resources of the node",
         "req": {"rdma": 25, "gpu-core": 50, "gpu-memory-ratio": 50},
         "node": node(gpu=[(0, GPU(1000, 1000, 160 * GI), GPU(25, 25, 4 * GI))], rdma=[(0, 1000, 50)]), "want": 184},
        {"src": "scoring_test.go:83-99", "name": "no device resources (a nodeDevice without devices)",
         "req": {"gpu-core": 100, "gpu-memory-ratio": 100}, "node": node(), "want": 0},
        {"src": "scoring_test.go:74-81", "name": "error missing nodecache (no nodeDevice entry)",
         "req": {"gpu-core": 100, "gpu-memory-ratio": 100}, "node": node(present=False), "want": 0},
    ],
    # scoring_test.go Test_resourceAllocationScorer_scoreDevice (one device)
    "score_device": [
        {"src": "scoring_test.go:1057-1069", "req": 50, "total": 100, "free": 100, "want": 50},
        {"src": "scoring_test.go:1070-1082", "req": 50, "total": 100, "free": 0, "want": 0},
        {"src": "scoring_test.go:1083-1095", "req": 30, "total": 100, "free": 50, "want": 20},
        {"src": "scoring_test.go:1096-1109", "req": 30, "total": 100, "free": 50, "most": True, "want": 80},
    ],
    # scoring_test.go TestScoreExtension (DefaultNormalizeScore)
    "normalize": [
        {"src": "scoring_test.go:512-526", "scores": [0], "want": [0]},
        {"src": "scoring_test.go:527-541", "scores": [10], "want": [100]},
        {"src": "scoring_test.go:542-564", "scores": [200, 10], "want": [100, 5]},
    ],
    # plugin_test.go Test_Plugin_Filter (pass = want nil)
    "filter": [
        {"src": "plugin_test.go:718-725", "name": "error missing nodecache", "req": {"gpu-core": 100, "gpu-memory-ratio": 100},
         "node": node(present=False), "pass": True},
        {"src": "plugin_test.go:726-743", "name": "insufficient device resource 1",
         "req": {"gpu-core": 100, "gpu-memory-ratio": 100}, "node": node(), "pass": False},
        {"src": "plugin_test.go:744-789", "name": "insufficient device resource 2",
         "req": {"gpu-core": 100, "gpu-memory-ratio": 100},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(25, 25, 4 * GI))]), "pass": False},
        {"src": "plugin_test.go:790-846", "name": "insufficient device resource 3",
         "req": {"fpga": 100, "gpu-core": 100, "gpu-memory-ratio": 100},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(25, 25, 4 * GI))], fpga=[(0, 100, 0)]), "pass": False},
        {"src": "plugin_test.go:847-908", "name": "insufficient device resource 4",
         "req": {"fpga": 100, "gpu-core": 100, "gpu-memory-ratio": 100},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(25, 25, 4 * GI))], fpga=[(0, 100, 50)]), "pass": False},
        {"src": "plugin_test.go:909-941", "name": "sufficient device resource 1", "req": {"fpga": 100},
         "node": node(fpga=[(0, 100, 0)]), "pass": True},
        {"src": "plugin_test.go:942-986", "name": "sufficient device resource 2", "req": {"fpga": 100},
         "node": node(fpga=[(0, 100, 25), (1, 100, 0)]), "pass": True},
        {"src": "plugin_test.go:987-1034", "name": "sufficient device resource 3",
         "req": {"gpu-core": 100, "gpu-memory-ratio": 100},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(0, 0, 0))], fpga=[(0, 100, 0)]), "pass": True},
        {"src": "plugin_test.go:1035-1090", "name": "sufficient device resource 4",
         "req": {"gpu-core": 100, "gpu-memory-ratio": 100},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(75, 75, 12 * GI)), (1, GPU(100, 100, 16 * GI), GPU(0, 0, 0))]),
         "pass": True},
        {"src": "plugin_test.go:1091-1145", "name": "sufficient device resource 5", "req": {"gpu-memory-ratio": 100},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(75, 75, 12 * GI)), (1, GPU(100, 100, 16 * GI), GPU(0, 0, 0))]),
         "pass": True},
        {"src": "plugin_test.go:1146-1200", "name": "sufficient device resource 6", "req": {"gpu-memory": 16 * GI},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(75, 75, 12 * GI)), (1, GPU(100, 100, 16 * GI), GPU(0, 0, 0))]),
         "pass": True},
    ],
    # plugin_test.go Test_Plugin_Reserve: ok + the allocated minors per type and
    # the used amounts after (plugin_test.go:1573-2400)
    "reserve": [
        {"src": "plugin_test.go:1605-1654", "name": "insufficient device resource 1",
         "req": {"gpu-core": 100, "gpu-memory-ratio": 100},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(75, 75, 12 * GI))]), "ok": False},
        {"src": "plugin_test.go:1655-1704", "name": "insufficient device resource 2",
         "req": {"gpu-core": 200, "gpu-memory-ratio": 200},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(75, 75, 12 * GI))]), "ok": False},
        {"src": "plugin_test.go:1705-1746", "name": "insufficient device resource 3",
         "req": {"gpu-core": 200, "gpu-memory-ratio": 200},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(0, 0, 0))]), "ok": False},
        {"src": "plugin_test.go:1747-1789", "name": "insufficient device resource 4", "req": {"rdma": 100},
         "node": node(rdma=[(0, 100, 50)]), "ok": False},
        {"src": "plugin_test.go:1790-1837", "name": "insufficient device resource 5", "req": {"rdma": 200, "fpga": 200},
         "node": node(rdma=[(0, 100, 0)], fpga=[(0, 100, 0)]), "ok": False},
        {"src": "plugin_test.go:1838-1991", "name": "sufficient device resource 1",
         "req": {"rdma": 100, "fpga": 100, "gpu-core": 100, "gpu-memory-ratio": 100},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(0, 0, 0))], rdma=[(0, 100, 0)], fpga=[(0, 100, 0)]),
         "ok": True, "minors": {"gpu": [0], "rdma": [0], "fpga": [0]},
         "used": {"gpu": {"0": GPU(100, 100, 16 * GI)}, "rdma": {"0": 100}, "fpga": {"0": 100}}},
        {"src": "plugin_test.go:1992-2221", "name": "sufficient device resource 2",
         "req": {"rdma": 200, "fpga": 200, "gpu-core": 200, "gpu-memory-ratio": 200},
         "node": node(gpu=[(0, GPU(100, 100, 16 * GI), GPU(0, 0, 0)), (1, GPU(100, 100, 16 * GI), GPU(0, 0, 0))],
                      rdma=[(0, 100, 0), (1, 100, 0)], fpga=[(0, 100, 0), (1, 100, 0)]),
         "ok": True, "minors": {"gpu": [0, 1], "rdma": [0, 1], "fpga": [0, 1]},
         "used": {"gpu": {"0": GPU(100, 100, 16 * GI), "1": GPU(100, 100, 16 * GI)}, "rdma": {"0": 100, "1": 100},
                  "fpga": {"0": 100, "1": 100}}},
    ],
    # utils_test.go: ValidateDeviceRequest (want: combination bits; error), ConvertDeviceRequest,
    # isPodRequestsMultipleDevice, memoryRatioToBytes / memoryBytesToRatio, fillGPUTotalMem
    "validate": [
        {"src": "utils_test.go:37-42", "req": {}, "err": True},
        {"src": "utils_test.go:43-50", "req": {"koordinator.sh/gpu-core": 101}, "err": True},
        {"src": "utils_test.go:51-62", "req": {"nvidia.com/gpu": 2, "koordinator.sh/gpu": 200,
                                               "koordinator.sh/gpu-core": 200, "koordinator.sh/gpu-memory": 32 * GI,
                                               "koordinator.sh/gpu-memory-ratio": 200}, "err": True},
        {"src": "utils_test.go:63-70", "req": {"koordinator.sh/gpu": 101}, "err": True},
        {"src": "utils_test.go:71-79", "req": {"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 101},
         "err": True},
        {"src": "utils_test.go:80-87", "req": {"nvidia.com/gpu": 2}, "want": 1},
        {"src": "utils_test.go:88-95", "req": {"dcu.com/gpu": 2}, "want": 2},
        {"src": "utils_test.go:96-103", "req": {"koordinator.sh/gpu": 200}, "want": 4},
        {"src": "utils_test.go:104-112", "req": {"koordinator.sh/gpu-core": 200, "koordinator.sh/gpu-memory": 64 * GI},
         "want": 8 | 16},
        {"src": "utils_test.go:113-121", "req": {"koordinator.sh/gpu-core": 200, "koordinator.sh/gpu-memory-ratio": 200},
         "want": 8 | 32},
        {"src": "utils_test.go:122-129", "req": {"koordinator.sh/gpu-memory-ratio": 200}, "want": 32},
        {"src": "utils_test.go:130-137", "req": {"koordinator.sh/gpu-memory": 64 * GI}, "want": 16},
        {"src": "utils_test.go:138-145", "req": {"koordinator.sh/fpga": 201}, "err": True},
        {"src": "utils_test.go:146-153", "req": {"koordinator.sh/fpga": 50}, "want": 64},
        {"src": "utils_test.go:154-161", "req": {"koordinator.sh/rdma": 201}, "err": True},
        {"src": "utils_test.go:162-169", "req": {"koordinator.sh/rdma": 50}, "want": 128},
    ],
    "convert": [
        {"src": "utils_test.go:210-222", "req": {"nvidia.com/gpu": 2}, "comb": 1,
         "want": {"koordinator.sh/gpu-core": 200, "koordinator.sh/gpu-memory-ratio": 200}},
        {"src": "utils_test.go:223-235", "req": {"dcu.com/gpu": 2}, "comb": 2,
         "want": {"koordinator.sh/gpu-core": 200, "koordinator.sh/gpu-memory-ratio": 200}},
        {"src": "utils_test.go:236-248", "req": {"koordinator.sh/gpu": 50}, "comb": 4,
         "want": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}},
        {"src": "utils_test.go:249-262", "req": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50},
         "comb": 8 | 32, "want": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}},
        {"src": "utils_test.go:263-276", "req": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory": 32 * GI},
         "comb": 8 | 16, "want": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory": 32 * GI}},
        {"src": "utils_test.go:277-288", "req": {"koordinator.sh/rdma": 80}, "comb": 128, "want": {"koordinator.sh/rdma": 80}},
        {"src": "utils_test.go:289-300", "req": {"koordinator.sh/fpga": 80}, "comb": 64, "want": {"koordinator.sh/fpga": 80}},
    ],
    # fillGPUTotalMem through the Filter of one GPU: the filled request must fit
    # exactly one device of the given free amounts (utils_test.go:431-506; the
    # memory conversions :415-429)
    "fill": [
        {"src": "utils_test.go:444-461", "total_mem": 32 * GI, "req": {"gpu-core": 50, "gpu-memory-ratio": 50},
         "want": {"gpu-core": 50, "gpu-memory-ratio": 50, "gpu-memory": 16 * GI}},
        {"src": "utils_test.go:462-480", "total_mem": 32 * GI, "req": {"gpu-core": 50, "gpu-memory": 16 * GI},
         "want": {"gpu-core": 50, "gpu-memory-ratio": 50, "gpu-memory": 16 * GI}},
        {"src": "utils_test.go:415-421", "total_mem": 64 * GI, "req": {"gpu-memory-ratio": 50},
         "want": {"gpu-core": 0, "gpu-memory-ratio": 50, "gpu-memory": 32 * GI}},
        {"src": "utils_test.go:423-429", "total_mem": 64 * GI, "req": {"gpu-memory": 32 * GI},
         "want": {"gpu-core": 0, "gpu-memory-ratio": 50, "gpu-memory": 32 * GI}},
    ],
    "multiple": [
        {"src": "utils_test.go:328-337", "type": "gpu", "req": {"gpu-memory-ratio": 100}, "want": False},
        {"src": "utils_test.go:338-347", "type": "fpga", "req": {"fpga": 300}, "want": True},
        {"src": "utils_test.go:348-357", "type": "fpga", "req": {"fpga": 30}, "want": False},
        {"src": "utils_test.go:358-367", "type": "rdma", "req": {"rdma": 300}, "want": True},
        {"src": "utils_test.go:368-377", "type": "rdma", "req": {"rdma": 30}, "want": False},
        {"src": "utils_test.go:386-395", "type": "gpu", "req": {"gpu-memory-ratio": 80}, "want": False},
        {"src": "utils_test.go:396-405", "type": "gpu", "req": {"gpu-memory-ratio": 200}, "want": True},
    ],
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "deviceshare_cases.json")
    json.dump(CASES, open(out, "w"), indent=1)
    print(out)

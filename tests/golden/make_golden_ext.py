"""Generates tests/golden/ext.json: reference test vectors of the Reservation and DeviceShare plugins (SURVEY 8(f)
rank 2), transcribed by hand from the reference's Go test tables into data (quantities in the ABI units: cpu milli,
memory / gpu-memory bytes, gpu-core and gpu-memory-ratio in percent units).

  reservation/scoring_test.go:40-253      TestScore (PreScore + Score through NominateReservation)
  reservation/scoring_test.go:255-390     TestScoreWithOrder (reservation-order label, mostPreferredScore, NormalizeScore)
  deviceshare/scoring_test.go:40-506      TestScore (GPU cases; the RDMA, preemptible and reserved cases are outside
                                          the device path's GPU-only scope and are not transcribed)
  deviceshare/scoring_test.go:1092-1167   Test_resourceAllocationScorer_scoreDevice

    python tests/golden/make_golden_ext.py
"""
import json
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ext.json")
Gi = 1 << 30


def main():
    reservation_score = [
        # the test node has an empty Status (Allocatable 0), no pods; nodeRState.podRequested / rAllocated unset
        {"name": "no reservation matched on the node", "src": "reservation/scoring_test.go:120-125",
         "pod": {"cpu": 0, "memory": 0, "keys": []}, "reservations": [], "want": 0},
        {"name": "reservation matched but zero-request pod", "src": "reservation/scoring_test.go:126-133",
         "pod": {"cpu": 0, "memory": 0, "keys": []},
         "reservations": [{"cpu": 2000, "memory": 4 * Gi}], "want": 0},
        {"name": "reservation matched and pod has part empty resource requests", "src": "reservation/scoring_test.go:134-154",
         "pod": {"cpu": 2000, "memory": 4 * Gi, "keys": ["cpu", "memory"]},
         "reservations": [{"cpu": 4000, "memory": 8 * Gi}], "want": 50},
        {"name": "allocated reservation matched and pod has part empty resource requests",
         "src": "reservation/scoring_test.go:155-181",
         "pod": {"cpu": 2000, "memory": 4 * Gi, "keys": ["cpu", "memory"]},
         "reservations": [{"cpu": 2000, "memory": 4 * Gi, "allocated": {"cpu": 2000, "memory": 3 * Gi}}], "want": 0},
        {"name": "multi reservations matched and pod has part empty resource requests",
         "src": "reservation/scoring_test.go:182-203",
         "pod": {"cpu": 2000, "memory": 4 * Gi, "keys": ["cpu", "memory"]},
         "reservations": [{"cpu": 4000, "memory": 8 * Gi}, {"cpu": 2000, "memory": 4 * Gi}], "want": 100},
    ]
    reservation_order = {
        "src": "reservation/scoring_test.go:255-390",
        "pod": {"cpu": 4000, "memory": 8 * Gi, "keys": ["cpu", "memory"]},
        # one 4C8G reservation per node; the 4th carries reservation-order 123456
        "orders": [0, 0, 0, 123456],
        "reservation": {"cpu": 4000, "memory": 8 * Gi},
        "want_preferred": 3,
        "want_scores": [100, 100, 100, 1000],
        "want_normalized": [10, 10, 10, 100],
    }
    gpu16 = {"core": 100, "ratio": 100, "memory": 16 * Gi}
    device_score = [
        {"name": "no device resources", "src": "deviceshare/scoring_test.go:95-113",
         "request": {"core": 100, "ratio": 100}, "gpus": None, "want": 0},
        {"name": "completely idle node", "src": "deviceshare/scoring_test.go:114-143",
         "request": {"core": 100, "ratio": 100}, "gpus": [{"minor": 0, "total": gpu16, "used": None}], "want": 0},
        {"name": "multiple GPU devices and completely idle", "src": "deviceshare/scoring_test.go:144-182",
         "request": {"core": 50, "ratio": 50},
         "gpus": [{"minor": 0, "total": gpu16, "used": None}, {"minor": 1, "total": gpu16, "used": None}], "want": 75},
        {"name": "remaining device resources", "src": "deviceshare/scoring_test.go:183-227",
         "request": {"core": 50, "ratio": 50},
         "gpus": [{"minor": 0, "total": gpu16, "used": {"core": 25, "ratio": 25, "memory": 4 * Gi}}], "want": 25},
        {"name": "remaining device resources with MostAllocated strategy", "src": "deviceshare/scoring_test.go:228-273",
         "strategy": "MostAllocated", "request": {"core": 50, "ratio": 50},
         "gpus": [{"minor": 0, "total": gpu16, "used": {"core": 25, "ratio": 25, "memory": 4 * Gi}}], "want": 75},
    ]
    score_device = [   # scoreDevice with the default args (weights: gpu-memory-ratio 1)
        {"name": "completely idle", "src": "deviceshare/scoring_test.go:1101-1113",
         "request": {"ratio": 50}, "total": {"ratio": 100}, "free": {"ratio": 100}, "want": 50},
        {"name": "completely used", "src": "deviceshare/scoring_test.go:1114-1126",
         "request": {"ratio": 50}, "total": {"ratio": 100}, "free": {"ratio": 0}, "want": 0},
        {"name": "remaining resources", "src": "deviceshare/scoring_test.go:1127-1139",
         "request": {"ratio": 30}, "total": {"ratio": 100}, "free": {"ratio": 50}, "want": 20},
        {"name": "remaining resources with MostAllocated", "src": "deviceshare/scoring_test.go:1140-1153",
         "strategy": "MostAllocated", "request": {"ratio": 30}, "total": {"ratio": 100}, "free": {"ratio": 50},
         "want": 80},
    ]
    with open(OUT, "w") as f:
        json.dump({"reservation_score": reservation_score, "reservation_order": reservation_order,
                   "device_score": device_score, "score_device": score_device}, f, indent=1)
    print(OUT)


if __name__ == "__main__":
    main()

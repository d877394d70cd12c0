import sys, os, json
sys.path.insert(0, os.getcwd())
import bench, torch
dev = torch.device("cuda:0")
for shp in [(16, 2048, 2048), (2, 512, 512), (32, 2000, 1000), (8, 4096, 4096)]:
    r = bench.chamfer_rate(dev, *shp)
    print(json.dumps({k: r[k] for k in ("shape", "ms", "gpair_dist_s", "path")}))

import ctypes, os, sys
import torch  # load torch's HIP runtime first, as the product path does
torch.cuda.init()
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgraph_probe.so"))
sys.exit(lib.graph_probe())

import torch, sys
a = torch.load(sys.argv[1], weights_only=True); b = torch.load(sys.argv[2], weights_only=True)
print("grad bitwise:", torch.equal(a["grad"], b["grad"]), "loss bitwise:", torch.equal(a["loss"], b["loss"]))

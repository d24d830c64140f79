import os, sys
sys.path.insert(0, "/root/repo")
import quest_amd as qa
from quest_amd.ops import capi
env = qa.Env()
reg = qa.Register(env, 20)
reg.init_plus()
for q in range(20): reg.z(q)
reg.sync()
print("ok")

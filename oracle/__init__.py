"""CPU oracle for the batched physics step — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package. The product path (mujoco_gymnasium_environments_amd) never does.
"""

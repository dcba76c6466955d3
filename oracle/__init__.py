"""ORACLE / TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference's ParkingModel hot path, used solely as the checker by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product package
(e2e-parking-carla_amd/) never imports, links or executes anything under oracle/.
"""

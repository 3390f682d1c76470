"""Copy the reference's saved MO trajectory of KITTI 2011_10_03_drive_0042 (a data file the
reference holds: src/vloam_main/results/2011_10_03_drive_0042/MO1.txt, 539 rows written by
vloam_tf.cpp:136-160) into tests/golden/kitti_mo1_2011_10_03_0042.txt, the fixture of
tests/test_trajectory.py.  Run here (the reference is not on the GPU box)."""
import os
import shutil

SRC = "/root/reference/src/vloam_main/results/2011_10_03_drive_0042/MO1.txt"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kitti_mo1_2011_10_03_0042.txt")

if __name__ == "__main__":
    shutil.copyfile(SRC, DST)
    print(DST)

"""Experiment drivers with the structure of the reference's test*.py
(module-level config globals, ``worker(fold, n_users, n_items, dataset_dir)``,
mean/std over folds).  Run e.g.::

    python -m collaborativefilteringusingtensorflow_amd.drivers.testbprmf <dataset_dir> [folds]
"""

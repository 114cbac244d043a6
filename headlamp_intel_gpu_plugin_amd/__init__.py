"""MI355X-native Headlamp GPU-observability plugin — Python tooling.

The shipped artefact is the Headlamp plugin (``src/``, JavaScript/TSX). This
package holds everything around it that runs outside the browser:

* ``models``   — synthetic MI355X clusters and their telemetry;
* ``sim``      — fake kube-apiserver + PromQL-subset Prometheus;
* ``ops``      — native C++/HIP code: the MI355X telemetry probe / exporter
                 and the GPU workload kernels synthetic pods run;
* ``parallel`` — one-process-per-GPU launch helpers for the benchmark;
* ``utils``    — statistics and the Node.js bridge.
"""
__version__ = "0.6.0"

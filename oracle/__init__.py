"""CPU oracle for the sbod hot path — TEST INFRASTRUCTURE ONLY.

A from-scratch CPU restatement of the reference's algorithms (each function cites the
reference file:line it follows).  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it, and only as the checker / the timed CPU
baseline — never as the product path.  The product package ``shape_based_object_detection_amd``
never imports this module and raises if its HIP library is missing.

Pinning: every function here is checked against golden fixtures produced by running the
reference itself (``tests/golden/make_golden.py``; ``tests/test_oracle_golden.py``).
The one third-party boundary — ``torchvision.ops.nms`` (absent from this image, version
unpinned) — is pinned through the reference's own ``operators.iou_utils.nms`` as SURVEY.md
§8(c) prescribes; see ``match_ref.nms_greedy``.

Modules:
  * ``match_ref``  — numpy: pairwise IoU, anchor matching, box codecs, greedy NMS, detect.
  * ``loss_ref``   — torch-CPU fp32 with autograd: the loss family and the criteria.
  * ``dcn_ref``    — torch-CPU fp32 with autograd: DeformConv2d (modulated, border-clamped).
"""

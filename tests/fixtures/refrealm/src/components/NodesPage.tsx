import React from 'react';
import { SectionBox, SimpleTable } from '@kinvolk/headlamp-plugin/lib/CommonComponents';
import { useIntelGpuContext } from '../api/IntelGpuDataContext';

// Fixture page: the header the bench waits for and one row per GPU node.
export default function NodesPage() {
  const { gpuNodes, gpuPods } = useIntelGpuContext();
  return (
    <SectionBox title="Intel GPU — Nodes">
      <SimpleTable columns={[{ label: 'Node', getter: (n: any) => n.metadata.name }]} data={gpuNodes} />
      <p>{gpuPods.length} pods</p>
    </SectionBox>
  );
}
